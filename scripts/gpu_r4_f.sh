#!/bin/bash
# After dropping the fused user kernels (slower), M-aware GEMM dispatch, Adam step counter in the
# cast launch: tests, bench, kernel profile, and a HIP API + memory-copy trace of the step seam.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_f 600 $T tests/test_step_graph.py tests/test_user_step_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_text_head_gpu.py -k "graph or user or gemm or linear or engine or head or adam or cast"
run bench 300 python -u bench.py
O=$PWD/gpurun_out/prof_c2f
rm -rf $O; mkdir -p $O
run prof_c2f 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_f.json > gpurun_out/breakdown_c2f.txt 2>&1
python benchmarks/phase_breakdown.py "$f" --until sample_kernel --json gpurun_out/r4_cache_build_f.json > gpurun_out/cache_build_f.txt 2>&1
head -30 gpurun_out/breakdown_c2f.txt
head -10 gpurun_out/cache_build_f.txt
O=$PWD/gpurun_out/prof_seam
rm -rf $O; mkdir -p $O
run prof_seam 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O -o s -- python -u bench.py --steps 12 --warmup 5 --round off --no-valid
ls $O
