#!/bin/bash
# where the timed window's fixed overhead goes: per-step device events, warm-up length
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
export FEDREC_BENCH_EVENTS=1
run r5ac_w5a 200 python -u bench.py --steps 20 --warmup 5 --round off --no-valid
run r5ac_w5b 200 python -u bench.py --steps 20 --warmup 5 --round off --no-valid
run r5ac_w30 200 python -u bench.py --steps 20 --warmup 30 --round off --no-valid
run r5ac_s50 200 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
