#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run multirank2 1000 python -u -m pytest tests/test_multirank_gpu.py -x -v -m gpu --timeout 700 --timeout-method thread
