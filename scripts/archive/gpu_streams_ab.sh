#!/bin/bash
# A/B: backbone on 1 vs 2 streams (two title halves interleaved by layer), same box.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run t_pack 300 python -u -m pytest tests/test_packed_gpu.py -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  FEDREC_BACKBONE_STREAMS=1 run s1_$r 300 python bench.py --steps 30 --warmup 5 --no-valid
  FEDREC_BACKBONE_STREAMS=2 run s2_$r 300 python bench.py --steps 30 --warmup 5 --no-valid
done
FEDREC_BACKBONE_STREAMS=2 run t_pack2 300 python -u -m pytest tests/test_packed_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread
