#!/bin/bash
# wave-state + utilisation counters of the current config-2 step (each pass its own run)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/pmc_r5v
rm -rf "$O"; mkdir -p "$O"
B="python -u bench.py --steps 20 --warmup 5 --round off --no-valid"
run pmc_v1 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC -- $B
run pmc_v2 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s2 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES -- $B
run pmc_v3 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p1 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- $B
run pmc_v4 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p2 --pmc FETCH_SIZE TCC_HIT_sum -- $B
run pmc_v5 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p3 --pmc WRITE_SIZE TCC_MISS_sum -- $B
for p in p1 p2 p3; do f=$(find "$O" -name "*${p}_counter_collection.csv" | head -1); [ -n "$f" ] && [ "$f" != "$O/${p}_counter_collection.csv" ] && cp "$f" "$O/${p}_counter_collection.csv"; done
python benchmarks/pmc_stalls.py "$O" > gpurun_out/r5_pmc_stalls_step_final.json
python benchmarks/pmc_summary.py "$O" > gpurun_out/r5_pmc_step_cfg2_final.json
echo done
