#!/bin/bash
# round-6 evidence on the current tree: configs 3 / 4 / 5 (driver default), config 2 at 50 steps,
# then per-kernel counters of the config-2 bench (each pass its own run)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r6t_c2_50 200 python -u bench.py --gpus 1 --steps 50 --warmup 10 --no-probe
run r6t_c3 200 python -u bench.py --config 3
run r6t_c4 200 python -u bench.py --config 4
run r6t_c5 400 python -u bench.py --config 5
O=$PWD/gpurun_out/pmc_r6t
rm -rf "$O"; mkdir -p "$O"
B="python -u bench.py --steps 20 --warmup 5 --round off --no-valid"
run pmc_t1 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC -- $B
run pmc_t2 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s2 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES -- $B
run pmc_t3 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p1 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- $B
run pmc_t4 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p2 --pmc FETCH_SIZE TCC_HIT_sum -- $B
run pmc_t5 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p3 --pmc WRITE_SIZE TCC_MISS_sum -- $B
for p in s1 s2 p1 p2 p3; do f=$(find "$O" -name "*${p}_counter_collection.csv" | head -1); [ -n "$f" ] && [ "$f" != "$O/${p}_counter_collection.csv" ] && cp "$f" "$O/${p}_counter_collection.csv"; done
python benchmarks/pmc_stalls.py "$O" > gpurun_out/r6_pmc_stalls_step_final.json
python benchmarks/pmc_summary.py "$O" > gpurun_out/r6_pmc_step_cfg2_final.json
grep -h -o '"value": [0-9.]*\|"steady_ms_per_step": [0-9.]*\|"baseline_config": [0-9]' gpurun_out/r6t_c*.log
head -c 1500 gpurun_out/r6_pmc_step_cfg2_final.json
