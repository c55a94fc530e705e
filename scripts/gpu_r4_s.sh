#!/bin/bash
# DMA-aware split-K: small-GEMM + user-step + step-graph tests, bench.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_s 600 $T tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py
run bench 300 python -u bench.py
run bench50 300 python -u bench.py --steps 50
