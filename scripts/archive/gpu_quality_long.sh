#!/bin/bash
# 10-epoch quality run (plain-CE scorer, lr 1e-4, GA, 1 client, planted-signal mind-small).
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/q
run q_long 1100 python Gradient_Averaging_main.py 10 64 5 --data_dir=synthetic:mind-small --lr=1e-4 \
    --score_act=identity --metrics_path=gpurun_out/q/ga_identity_lr1e-4_10ep.jsonl --snapshot_path=/tmp/ql/s.pt
