#!/bin/bash
# cache-build chunk size (the backbone GEMMs' M regime) + where the step's device copy comes from
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
for c in 8192 4096 2048 1600 8192; do
  run r5l_chunk_$c 200 env FEDREC_CACHE_CHUNK=$c python -u bench.py --round off --no-valid --steps 5 --warmup 2
done
