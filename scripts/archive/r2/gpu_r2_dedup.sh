#!/bin/bash
# 32-bit-key dedup + 3-stage wgrad: tests, wgrad stage A/B, config-2 bench + profile
source "$(dirname "$0")/../../gpu_lib.sh"
check ktests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_wgrad_gpu.py tests/test_engine_gpu.py tests/test_user_step_gpu.py -m gpu
FEDREC_WGRAD_NST=4 run bwd4 300 python benchmarks/bwd_gemm_bench.py --rounds 5
run bwd3 300 python benchmarks/bwd_gemm_bench.py --rounds 5
run bench 400 python bench.py --steps 50 --warmup 10
O=$PWD/gpurun_out/prof_dd
rm -rf $O; mkdir -p $O
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
