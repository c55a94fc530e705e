"""Where the gradient all-reduce launches sit in an N > 1 step (rocprofv3 kernel trace of ONE
client process): for each step (between two in-graph Adam kernels) the start of every IPC
all-reduce launch relative to the text head's backward kernels.  With the early user-slice
reduce the first all-reduce starts before ``head_pool_bwd3`` / ``head_wgrad_g`` and runs beside
them; the second (text-head slice) after ``head_reduce``.

    python benchmarks/early_reduce_order.py trace.csv [--json out.json]
"""
import argparse
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--json", default="")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "adam_dev" in r["Kernel_Name"]]
steps = []
for i0, i1 in zip(marks, marks[1:]):
    t0 = int(rows[i0]["End_Timestamp"])
    ev = {}
    for r in rows[i0 + 1:i1 + 1]:
        n = r["Kernel_Name"]
        key = ("ipc_allreduce" if "ipc_allreduce" in n else "head_pool_bwd" if "head_pool_bwd" in n else
               "head_wgrad_g" if "head_wgrad_g" in n else "head_reduce" if "head_reduce" in n else
               "adam" if "adam_dev" in n else None)
        if key is None:
            continue
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        ev.setdefault(key, []).append((round(s, 1), round(e, 1), r.get("Stream_Id", "")))
    steps.append(ev)
out = []
for ev in steps:
    ar = ev.get("ipc_allreduce", [])
    wg = ev.get("head_wgrad_g", [(None, None, None)])[0]
    pb = ev.get("head_pool_bwd", [(None, None, None)])[0]
    out.append({"allreduce_us": ar, "head_pool_bwd_us": pb, "head_wgrad_g_us": wg,
                "head_reduce_us": ev.get("head_reduce", [None])[0],
                "first_allreduce_before_wgrad": bool(ar and wg[0] is not None and ar[0][0] < wg[0])})
for o in out[-6:]:
    print(json.dumps(o))
n_ok = sum(o["first_allreduce_before_wgrad"] for o in out)
print(f"steps {len(out)}: first all-reduce launched before head_wgrad_g in {n_ok}")
if a.json:
    json.dump({"steps": out, "early_before_wgrad": n_ok}, open(a.json, "w"), indent=1)
