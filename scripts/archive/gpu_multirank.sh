#!/bin/bash
# two client processes sharing the GPU (gloo data plane), then the GPU suite and the config-2 bench
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run multirank 600 python -u -m pytest tests/test_multirank_gpu.py -x -v -m gpu --timeout 450 --timeout-method thread
run gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
run bench_cfg2 600 python bench.py --config 2 --steps 30 --warmup 5
