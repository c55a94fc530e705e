#!/bin/bash
# small-GEMM launch compositions / split-K probe; configs 3 and 4 benches.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run sgshapes 300 python -u benchmarks/sg_step_shapes.py gpurun_out/r4_sg_step_shapes_r.json
run bench_c3 300 python -u bench.py --config 3
run bench_c4 300 python -u bench.py --config 4
