#!/bin/bash
# N > 1: the text head's and fc's weight gradients written into the flat buffer by their backward
# launches -- multi-client tests (2 / 4 processes sharing the GPU), engine + head tests, and the
# early-reduce trace of two clients
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_v1 900 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 450 --timeout-method thread -p no:cacheprovider
check t_v2 600 python -u -m pytest tests/test_engine_gpu.py tests/test_text_head_gpu.py tests/test_step_fusions_gpu.py tests/test_deferred_reduce_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
grep -h "GRAPH_AR OK\|passed\|failed" gpurun_out/t_v1.log | tail -5
tail -2 gpurun_out/t_v2.log
