#!/bin/bash
# Small-GEMM LDS-DMA ring: kernel tests (bitwise vs the register-queue kernel), latency probe
# A/B (tile 5 vs 1), step tests, bench, step profile.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_sg 200 $T tests/test_small_gemm_gpu.py
run sgprobe 200 python -u benchmarks/sg_latency_probe.py gpurun_out/r4_sg_dma_probe.json
check t_j 500 $T tests/test_step_graph.py tests/test_engine_gpu.py tests/test_user_step_gpu.py
run bench 300 python -u bench.py
O=$PWD/gpurun_out/prof_c2j
rm -rf $O; mkdir -p $O
run prof_c2j 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_j.json > gpurun_out/breakdown_c2j.txt 2>&1
head -30 gpurun_out/breakdown_c2j.txt
