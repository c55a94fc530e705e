#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
rm -rf gpurun_out/quality_fed
run r5k_quality 900 python -u scripts/quality_fed.py --out gpurun_out/quality_fed --world 4 8
