#!/bin/bash
# Per-kernel PMC counters of a training step (three passes, each within one block's counter
# limits) for BASELINE config $1 (2: the headline; 4: LDP, the fused noise inside the captured
# step) plus its kernel trace / step breakdown.  Summaries: benchmarks/pmc_summary.py.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
CFG=${1:-2}
O=$PWD/gpurun_out/pmc_c$CFG
rm -rf "$O"; mkdir -p "$O"
B="python -u bench.py --config $CFG --steps 20 --warmup 5 --round off --no-valid"
run trace_c$CFG 300 rocprofv3 --kernel-trace --output-format csv -d "$O" -o tr -- $B
f=$(find "$O" -name "*tr_kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg${CFG}_step_breakdown.json > gpurun_out/breakdown_c$CFG.txt 2>&1
head -40 gpurun_out/breakdown_c$CFG.txt
run pmc_p1_c$CFG 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p1 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- $B
run pmc_p2_c$CFG 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p2 --pmc FETCH_SIZE TCC_HIT_sum -- $B
run pmc_p3_c$CFG 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p3 --pmc WRITE_SIZE TCC_MISS_sum -- $B
for p in p1 p2 p3; do f=$(find "$O" -name "*${p}_counter_collection.csv" | head -1); [ -n "$f" ] && [ "$f" != "$O/${p}_counter_collection.csv" ] && cp "$f" "$O/${p}_counter_collection.csv"; done
python benchmarks/pmc_summary.py "$O" > gpurun_out/r4_pmc_step_cfg$CFG.json
head -c 2000 gpurun_out/r4_pmc_step_cfg$CFG.json
