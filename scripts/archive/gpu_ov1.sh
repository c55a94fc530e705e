#!/bin/bash
# N = 1: Adam on the side stream (overlapping the next backbone) vs on the main stream
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
for i in 1 2; do
  run o1_$i 300 env FEDREC_OVERLAP_OPTIMIZER=on python bench.py --config 2 --steps 40 --warmup 5 --no-valid
  run o0_$i 300 env FEDREC_OVERLAP_OPTIMIZER=auto python bench.py --config 2 --steps 40 --warmup 5 --no-valid
done
grep -h '^{' gpurun_out/o1_*.log gpurun_out/o0_*.log > gpurun_out/ov1_ab.jsonl || true
