#!/bin/bash
# DMA ring stage counts + the step's small GEMMs standalone in their current / candidate forms.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_sg 200 $T tests/test_small_gemm_gpu.py
run sgshapes 300 python -u benchmarks/sg_step_shapes.py gpurun_out/r4_sg_step_shapes.json
