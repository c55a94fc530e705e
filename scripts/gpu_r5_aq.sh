#!/bin/bash
# config 5: per-step device intervals (is there a one-off inside the timed window?)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
export FEDREC_BENCH_EVENTS=1
run r5aq_c5_20 300 python -u bench.py --config 5 --steps 20 --warmup 5 --round off --no-valid
run r5aq_c5_10 300 python -u bench.py --config 5 --steps 10 --warmup 3 --round off --no-valid
for f in gpurun_out/r5aq_*.log; do echo $f; grep -o '"per_step": \[[^]]*\]' $f; grep -o '"steady_ms_per_step": [0-9.]*' $f; done
