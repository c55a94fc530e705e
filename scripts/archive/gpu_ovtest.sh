#!/bin/bash
# the overlapped-optimizer equivalence test, repeated (flakiness check of its statistic)
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
T="python -u -m pytest tests/test_engine_gpu.py -q -m gpu --timeout 120 --timeout-method thread -k overlapped"
for i in 1 2 3 4 5; do run ov_$i 200 $T; done
