"""Kernel time of one phase of a run from a rocprofv3 kernel trace (``--kernel-trace
--output-format csv``): every launch before the first launch of ``--until`` (default: the
device sampler, i.e. the hidden-state cache build that precedes the first training step),
grouped by kernel name, with the phase's wall span.

    python benchmarks/phase_breakdown.py gpurun_out/prof_c2/.../c2_kernel_trace.csv --until sample_kernel
"""
import argparse
import collections
import csv
import json

from step_breakdown import short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--until", default="sample_kernel")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    stop = next((e[0] for e in ev if a.until in e[2]), None)
    win = [e for e in ev if stop is None or e[0] < stop]
    per = collections.defaultdict(float)
    calls = collections.Counter()
    for s, e, n in win:
        per[short(n)] += (e - s) / 1e3
        calls[short(n)] += 1
    span = (win[-1][1] - win[0][0]) / 1e3 if win else 0.0
    busy = sum(per.values())
    out = {"span_us": round(span, 1), "kernel_sum_us": round(busy, 1),
           "kernels": [{"name": k, "us": round(v, 1), "launches": calls[k]}
                       for k, v in sorted(per.items(), key=lambda kv: -kv[1])]}
    print(f"phase span {span / 1e3:.2f} ms, kernel time {busy / 1e3:.2f} ms")
    for k in out["kernels"][:30]:
        print(f"  {k['us'] / 1e3:9.3f} ms  x{k['launches']:<5d} {k['name']}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
