#!/bin/bash
# Per-kernel PMC counters of the config-2 training step (three passes, each within one block's
# counter limits) + the text-head microbenchmark.  Summaries: benchmarks/pmc_summary.py.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/pmc_step
rm -rf "$O"; mkdir -p "$O"
B="python -u bench.py --steps 20 --warmup 5 --round off --no-valid"

run pmc_p1 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p1 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- $B
run pmc_p2 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p2 --pmc FETCH_SIZE TCC_HIT_sum -- $B
run pmc_p3 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p3 --pmc WRITE_SIZE TCC_MISS_sum -- $B
find "$O" -name "*counter_collection.csv" | head
for p in p1 p2 p3; do f=$(find "$O" -name "*${p}_counter_collection.csv" | head -1); [ -n "$f" ] && [ "$f" != "$O/${p}_counter_collection.csv" ] && cp "$f" "$O/${p}_counter_collection.csv"; done
python benchmarks/pmc_summary.py "$O" > gpurun_out/r3_pmc_step.json
head -c 3000 gpurun_out/r3_pmc_step.json
