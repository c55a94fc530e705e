"""One step's launches from a rocprofv3 kernel trace (between two consecutive marker kernels,
default the in-graph Adam): start offset, duration, queue / stream, name.

    python benchmarks/launch_seq.py trace.csv [--marker adam] [--back 2]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--marker", default="adam")
ap.add_argument("--back", type=int, default=2)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
i0, i1 = marks[-a.back - 1], marks[-a.back]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r.get("Stream_Id", r.get("Queue_Id", ""))
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  q={q:>3}  {r['Kernel_Name'][:100]}")
