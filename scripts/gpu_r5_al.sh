#!/bin/bash
# cache-build chunk: 13,000 titles (5 chunks, the 32-bit offset limit is ~13,981) vs 8,192 (8 chunks)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r5al_13k_1 200 env FEDREC_CACHE_CHUNK=13000 python -u bench.py --steps 20 --warmup 5 --round off --no-valid
run r5al_8k_1 200 env FEDREC_CACHE_CHUNK=8192 python -u bench.py --steps 20 --warmup 5 --round off --no-valid
run r5al_13k_2 200 env FEDREC_CACHE_CHUNK=13000 python -u bench.py --steps 20 --warmup 5 --round off --no-valid
run r5al_8k_2 200 env FEDREC_CACHE_CHUNK=8192 python -u bench.py --steps 20 --warmup 5 --round off --no-valid
run r5al_16k_1 200 env FEDREC_CACHE_CHUNK=16250 python -u bench.py --steps 20 --warmup 5 --round off --no-valid
for f in gpurun_out/r5al_*.log; do echo $f $(grep -o '"cache_build_ms": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f); done
