#!/bin/bash
# full GPU test suite, then the overlap test twice more (its statistic is run-to-run noise)
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run gputests 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -rf
for i in 1 2; do run overlap_rep$i 300 python -u -m pytest tests/test_engine_gpu.py -q -m gpu -k overlapped --timeout 120 --timeout-method thread; done
