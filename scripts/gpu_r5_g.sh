#!/bin/bash
# wave-state counters of the text-head kernels in isolation (benchmarks/head_bench.py)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/pmc_head
rm -rf "$O"; mkdir -p "$O"
B="python -u benchmarks/head_bench.py --iters 10"
run pmc_h1 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC -- $B
run pmc_h2 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s2 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES -- $B
run pmc_h3 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B
python benchmarks/pmc_stalls.py "$O" > gpurun_out/r5_pmc_stalls_head.json
python - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for p in glob.glob("gpurun_out/pmc_head/**/s3*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"].split("(")[0][-60:]
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, d in acc.items():
    if "head" in n:
        print(n, {k: round(v / 1e6, 3) for k, v in d.items()})
PY
