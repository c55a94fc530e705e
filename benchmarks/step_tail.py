"""The tail of each N > 1 step in a rocprofv3 kernel trace of ONE client process: the kernels
between the text head's reduce launch and the step's Adam, and the time from the end of
``head_reduce`` to the start of ``adam_dev``.  With the head's weight gradients written into the
flat buffer by their own launches the tail is [head slice all-reduce]; with the end-of-backward
copy it is [multi_cast, head slice all-reduce].  Groups the steps by their tail sequence.

    python benchmarks/step_tail.py trace.csv [--json out.json]
"""
import argparse
import collections
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--json", default="")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))


def short(n: str) -> str:
    for k in ("ipc_allreduce", "multi_cast", "adam", "copyBuffer", "splitk_reduce", "multi_copy"):
        if k in n:
            return k
    return n.split("(")[0][-40:]


groups = collections.defaultdict(list)
i = 0
while i < len(rows):
    if "head_reduce" in rows[i]["Kernel_Name"]:
        t0 = int(rows[i]["End_Timestamp"])
        seq = []
        j = i + 1
        while j < len(rows) and "adam" not in rows[j]["Kernel_Name"] and "head_reduce" not in rows[j]["Kernel_Name"]:
            seq.append(short(rows[j]["Kernel_Name"]))
            j += 1
        if j < len(rows) and "adam" in rows[j]["Kernel_Name"]:
            groups[" > ".join(seq)].append((int(rows[j]["Start_Timestamp"]) - t0) / 1e3)
        i = j
    else:
        i += 1
out = {k: {"steps": len(v), "mean_us_head_reduce_end_to_adam": round(sum(v) / len(v), 2)} for k, v in groups.items()}
print(json.dumps(out, indent=1))
if a.json:
    json.dump(out, open(a.json, "w"), indent=1)
