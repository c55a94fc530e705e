#!/bin/bash
# round-5 tree: configs 3 and 5 (driver default) + config 2 at 50 steps
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r5ab_c3 200 python -u bench.py --config 3
run r5ab_c5 400 python -u bench.py --config 5
run r5ab_c2_50 200 python -u bench.py --steps 50 --warmup 10
