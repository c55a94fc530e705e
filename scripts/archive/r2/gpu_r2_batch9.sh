#!/bin/bash
# small GEMM: two K-tiles in flight + split-K with the whole epilogue in the reduce
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py tests/test_engine_gpu.py tests/test_step_graph.py
run c2 300 python bench.py --steps 50 --warmup 10
run c2_default 300 python bench.py
O=$PWD/gpurun_out/prof_c2
rm -rf $O; mkdir -p $O
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
