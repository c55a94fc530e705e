"""Per-step kernel breakdown from a rocprofv3 kernel trace (``--kernel-trace --output-format
csv``): the window between the last ``--steps + 1`` launches of a step-marker kernel (default
the fused Adam), kernel time per step grouped by name, busy time vs step period.

    python benchmarks/step_breakdown.py gpurun_out/prof_full/c2_kernel_trace.csv --steps 10
"""
import argparse
import collections
import csv
import json
import re


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    m = re.match(r"([A-Za-z_0-9:]+(<[^()]*>)?)", name)
    return (m.group(1) if m else name)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="adam")  # adam_kernel (eager) or adam_dev_kernel (in the step graph)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    marks = [e for e in ev if a.marker in e[2]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker launches")
    t0, t1 = marks[-a.steps - 1][0], marks[-1][0]
    win = [e for e in ev if t0 <= e[0] < t1]
    per = collections.defaultdict(float)
    calls = collections.Counter()
    for s, e, n in win:
        per[short(n)] += (e - s) / 1e3 / a.steps
        calls[short(n)] += 1
    period = (t1 - t0) / 1e3 / a.steps
    busy = sum(per.values())
    out = {"period_us": round(period, 1), "kernel_sum_us": round(busy, 1),
           "kernels": [{"name": k, "us_per_step": round(v, 1), "launches_per_step": calls[k] / a.steps}
                       for k, v in sorted(per.items(), key=lambda kv: -kv[1])]}
    print(f"step period {period:.1f} us, kernel time {busy:.1f} us/step (both streams)")
    for k in out["kernels"]:
        print(f"  {k['us_per_step']:8.1f} us  x{k['launches_per_step']:<5g} {k['name']}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
