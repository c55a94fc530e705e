#!/bin/bash
# small-GEMM launch floor: kernel durations of shrinking launches (rocprofv3 kernel trace)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/prof_r5o
rm -rf $O; mkdir -p $O
run prof_r5o 200 rocprofv3 --kernel-trace --output-format csv -d $O -o p -- python -u benchmarks/sg_floor_probe.py
f=$(find $O -name "*kernel_trace.csv" | head -1)
python - "$f" <<'PY' > gpurun_out/r5o_floor.txt
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"][:60], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
# group consecutive launches of the same kernel name: 12 per (shape, tile)
groups, cur = [], []
for n, d in seq:
    if cur and (cur[0][0] != n or len(cur) == 12):
        groups.append(cur); cur = []
    cur.append((n, d))
groups.append(cur)
for g in groups:
    ds = sorted(d for _, d in g[2:])
    print(f"{g[0][0]:60s} n={len(g)} median={ds[len(ds)//2]:.2f} min={ds[0]:.2f} us")
PY
cat gpurun_out/r5o_floor.txt
