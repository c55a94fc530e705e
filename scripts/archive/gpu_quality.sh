#!/bin/bash
# Training-quality and FedAvg-round runs on one GPU (synthetic mind-small, random init):
#  * synchronous gradient averaging, 3 epochs, B=64 (1 client), plain-CE scoring (score_act=identity)
#  * star FedAvg: coordinator (rank 0, CPU) + 1 GPU client, 3 rounds x 1 local epoch
# (the reference's sigmoid-CE scorer (quirk Q1) saturates on random-init features: run 1 of
#  profiles/quality_r1_ga_sigmoid.jsonl stays at ln 5)
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/q
run q_ga 900 python Gradient_Averaging_main.py 3 64 1 --data_dir=synthetic:mind-small --score_act=identity \
    --metrics_path=gpurun_out/q/ga_identity.jsonl --snapshot_path=/tmp/q_ga.pt
run q_star 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29633 -m fedrec_with_pytorchdistributed_amd.cli star 3 1 64 --data_dir=synthetic:mind-small \
    --score_act=identity --metrics_path=gpurun_out/q/star_identity.jsonl --snapshot_path=/tmp/q_star.pt
