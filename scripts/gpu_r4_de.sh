#!/bin/bash
# Graph-replay seam micro; backbone GEMM correctness (bias-armed ping-pong v12 = auto, v13 NT)
# + A/B vs v9 and hipBLASLt; fused user fc1+pool fwd/bwd; step tests; bench + profiles.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
run gap 120 python -u benchmarks/graph_gap.py
check t_gemm 600 $T tests/test_kernels_gpu.py tests/test_wgrad_gpu.py tests/test_packed_gpu.py tests/test_gemm_partial_gpu.py -k "gemm or linear or pack or split or backbone or wgrad or upool_fc"
run gemm 400 python -u benchmarks/gemm_bench.py --rounds 5 --out gpurun_out/r4_gemm_bench.json
check t_d 500 $T tests/test_step_graph.py tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py tests/test_text_head_gpu.py tests/test_kernels_gpu.py -k "not gemm_variants"
run bench 300 python -u bench.py
O=$PWD/gpurun_out/prof_c2e
rm -rf $O; mkdir -p $O
run prof_c2e 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_e.json > gpurun_out/breakdown_c2e.txt 2>&1
python benchmarks/phase_breakdown.py "$f" --until sample_kernel --json gpurun_out/r4_cache_build_e.json > gpurun_out/cache_build_e.txt 2>&1
head -30 gpurun_out/breakdown_c2e.txt
head -12 gpurun_out/cache_build_e.txt
run gemm_big 400 python -u benchmarks/gemm_bench.py --rounds 3 --M 409600 --out gpurun_out/r4_gemm_bench_M409600.json
