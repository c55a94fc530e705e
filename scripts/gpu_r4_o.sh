#!/bin/bash
# bf16 operands from the user-side producers + the LDS-DMA ring for every bf16 small-GEMM launch
# (transposed operands, ones-MFMA column sums): tests, probe, bench, step profile.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
#check t_sg 300 $T tests/test_small_gemm_gpu.py
#check t_o 600 $T tests/test_user_step_gpu.py tests/test_kernels_gpu.py -k "user or small or score_ce or segment or pool"
check t_o2 600 $T tests/test_step_graph.py tests/test_engine_gpu.py tests/test_text_head_gpu.py
run sgshapes 300 python -u benchmarks/sg_step_shapes.py gpurun_out/r4_sg_step_shapes_o.json
run bench 300 python -u bench.py
run bench50 300 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_c2o
rm -rf $O; mkdir -p $O
run prof_c2o 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_o.json > gpurun_out/breakdown_c2o.txt 2>&1
head -32 gpurun_out/breakdown_c2o.txt
