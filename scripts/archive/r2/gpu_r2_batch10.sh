#!/bin/bash
# small GEMM back to one tile in flight (+ split-K with the full epilogue in the reduce);
# unroll-4 user-attention backward as variant 2: tests, micro A/B, config-2 A/B/A, profile
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py tests/test_kernels_gpu.py -k "small or user or gemm or colsum"
run uabench 200 python benchmarks/user_attn_bench.py --out gpurun_out/user_attn_bench.json
run c2_a 300 python bench.py --steps 50 --warmup 10
run c2_ua2 300 env FEDREC_UA_VARIANT=2 python bench.py --steps 50 --warmup 10
run c2_b 300 python bench.py --steps 50 --warmup 10
O=$PWD/gpurun_out/prof_c2
rm -rf $O; mkdir -p $O
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
