#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/q
run q_ga_lr 900 python Gradient_Averaging_main.py 4 64 1 --data_dir=synthetic:mind-small --score_act=identity --lr=1e-3 \
    --metrics_path=gpurun_out/q/ga_identity_lr1e-3.jsonl --snapshot_path=/tmp/q_ga2.pt
