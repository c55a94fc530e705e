#!/bin/bash
# A/B: device-memory kernel arguments (HIP_FORCE_DEV_KERNARG=1) vs the runtime default, A/B/A/B
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run ka0 300 python -u bench.py --steps 50
run kb1 300 env HIP_FORCE_DEV_KERNARG=1 python -u bench.py --steps 50
run ka2 300 python -u bench.py --steps 50
run kb3 300 env HIP_FORCE_DEV_KERNARG=1 python -u bench.py --steps 50
