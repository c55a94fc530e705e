#!/bin/bash
# Graph-replay seam micro + step profile after reverting the split-K seam and fixing the
# in-graph Adam / loss-sum costs.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run gap 120 python -u benchmarks/graph_gap.py
O=$PWD/gpurun_out/prof_gap
rm -rf $O; mkdir -p $O
run prof_gap 120 rocprofv3 --kernel-trace --output-format csv -d $O -o g -- python -u benchmarks/graph_gap.py
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_d 400 $T tests/test_step_graph.py tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py tests/test_text_head_gpu.py tests/test_kernels_gpu.py -k "not gemm_variants"
run bench 300 python -u bench.py
O=$PWD/gpurun_out/prof_c2d
rm -rf $O; mkdir -p $O
run prof_c2d 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_d.json > gpurun_out/breakdown_c2d.txt 2>&1
head -40 gpurun_out/breakdown_c2d.txt
