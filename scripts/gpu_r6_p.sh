#!/bin/bash
# star FedAvg at W = 4: the final global model with and without the server-step options
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run q_r6p 1100 python -u scripts/quality_fed.py --out gpurun_out/r6_quality_fed_w4 --world 4 --only 'star_w4$,star_w4_lr3m5,star_w4_m9,star_w4_lr3$'
cut -c1-400 gpurun_out/r6_quality_fed_w4/summary.jsonl
