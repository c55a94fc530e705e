#!/bin/bash
# bucketed (secure) gradient reduction during the backward; multi-client rehearsal on one GPU
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 1100 python -u -m pytest tests/test_multirank_gpu.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread
run bench_cfg5 600 python bench.py --config 5 --steps 20 --warmup 5
