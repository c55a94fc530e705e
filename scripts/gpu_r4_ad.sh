#!/bin/bash
# cache-build warm-up: the FIRST bench of a fresh box with the warm-up (default), then without, then with
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run w0 300 python -u bench.py
run n1 300 python -u bench.py --cache-warm 0
run w2 300 python -u bench.py
run n3 300 python -u bench.py --cache-warm 0
