#!/bin/bash
# bench with the learning probe (config 2 driver default; config 3 / 4 / 5)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r6j_c2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
run r6j_c3 300 python -u bench.py --config 3
run r6j_c4 300 python -u bench.py --config 4
run r6j_c5 400 python -u bench.py --config 5
for f in gpurun_out/r6j_*.log; do echo $f $(grep -o '"value": [0-9.]*\|"steady_ms_per_step": [0-9.]*\|"learning_probe": {[^}]*}\|"round_s": [0-9.]*\|"cache_build_ms": [0-9.]*' $f | tr '\n' ' '); done
