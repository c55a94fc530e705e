#!/bin/bash
# long-sequence (T > 64) title attention fwd/bwd + backbone forward vs the oracle
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run longtitle 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread -k "title_attention or long_titles"
