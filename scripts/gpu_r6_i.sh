#!/bin/bash
# server-step sweep 2 (W = 8): FedAdam for star, PA server lr 4 and K = 4
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run q_r6i 700 python -u scripts/quality_fed.py --out gpurun_out/r6_quality_fed3 --world 8 --only star_w8_adam,pa8_w8_mv_lr4,pa8_w8_k4
cut -c1-300 gpurun_out/r6_quality_fed3/summary.jsonl
