#!/bin/bash
# Held-batch events every 4 steps: tests, bench (driver default + 50 steps), step profile; then
# per-kernel counters of config 2 and config 4 (scripts/gpu_r4_pmc.sh).
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_i 500 $T tests/test_step_graph.py tests/test_engine_gpu.py tests/test_text_head_gpu.py tests/test_user_step_gpu.py
check t_ua 200 $T tests/test_kernels_gpu.py -k "user_attention or score_ce or segment"
run bench 300 python -u bench.py
run bench50 300 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_c2i
rm -rf $O; mkdir -p $O
run prof_c2i 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_i.json > gpurun_out/breakdown_c2i.txt 2>&1
head -8 gpurun_out/breakdown_c2i.txt
bash scripts/gpu_r4_pmc.sh 2
bash scripts/gpu_r4_pmc.sh 4
