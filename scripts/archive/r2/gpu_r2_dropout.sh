#!/bin/bash
# backbone dropout kernels vs the oracle, engine regressions, config-5 bench with dropout
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 900 python -u -m pytest tests/test_dropout.py tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_news_cache.py -x -q -m gpu --timeout 120 --timeout-method thread
run bench_cfg5 600 python bench.py --config 5 --steps 20 --warmup 5
