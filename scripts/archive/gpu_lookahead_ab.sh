#!/bin/bash
# GPU tests, then A/B of the batch lookahead stream (FEDREC_LOOKAHEAD=0 disables it), same box.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
for r in 1 2; do
  FEDREC_LOOKAHEAD=1 run la1_$r 300 python bench.py --steps 30 --warmup 5 --no-valid
  FEDREC_LOOKAHEAD=0 run la0_$r 300 python bench.py --steps 30 --warmup 5 --no-valid
done
