#!/bin/bash
# host profile of the step loop + federated quality at W = 4, 8 (shared GPU)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r5j_host 300 python -u benchmarks/host_profile.py --steps 300
run r5j_quality 900 python -u scripts/quality_fed.py --out gpurun_out/quality_fed --world 4 8
