#!/bin/bash
# round-5 opening tree: driver-default bench + 50-step arm (within-round reference)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r5_base_bench 300 python -u bench.py
run r5_base_bench50 300 python -u bench.py --steps 50
