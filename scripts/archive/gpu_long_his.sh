#!/bin/bash
# long-history (H > 64) user attention / pool kernels, oracle step with untruncated histories
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run longhis 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread -k "user_attention or additive_pool_long or oracle"
