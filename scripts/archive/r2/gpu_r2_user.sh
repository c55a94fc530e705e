#!/bin/bash
# fused device user side: oracle tests, engine regressions, bench, kernel stats
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 900 python -u -m pytest tests/test_user_step_gpu.py tests/test_small_gemm_gpu.py tests/test_engine_gpu.py tests/test_step_graph.py tests/test_news_cache.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread
run bench 300 python bench.py --steps 50 --warmup 10
O=$PWD/gpurun_out/prof_user
mkdir -p $O
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
