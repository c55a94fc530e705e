#!/bin/bash
# session-2 opening: driver-default bench + 50-step bench + step breakdown of the restored tree
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r5m_def 300 python -u bench.py
run r5m_50 300 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_r5m
rm -rf $O; mkdir -p $O
run prof_r5m 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r5_cfg2_step_breakdown_m.json > gpurun_out/breakdown_r5m.txt 2>&1
head -40 gpurun_out/breakdown_r5m.txt
python - "$f" <<'PY' > gpurun_out/r5m_launch_seq.txt
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
a, b = marks[-3], marks[-2]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  grid={r.get('Grid_Size','')} wg={r.get('Workgroup_Size','')} lds={r.get('LDS_Block_Size', r.get('Lds_Size',''))} vgpr={r.get('VGPR_Count', r.get('Arch_VGPR_Count',''))}  {r['Kernel_Name'][:110]}")
PY
