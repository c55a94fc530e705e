#!/bin/bash
# config 5: split-K target of the weight-gradient GEMMs (output tiles over all chunks)
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
for t in 512 256 1024 512; do
  run w$t 400 env FEDREC_WGRAD_TILES=$t python bench.py --config 5 --steps 10 --warmup 3 --no-valid
  grep -h '^{' gpurun_out/w$t.log | sed "s/^/$t /" >> gpurun_out/wgrad_ab.txt || true
done
