#!/bin/bash
# Training-quality and FedAvg-round runs on one GPU (synthetic mind-small, random init):
#  * synchronous gradient averaging, 3 epochs, B=64 (1 client)
#  * star FedAvg: coordinator (rank 0, CPU) + 1 GPU client, 3 rounds x 1 local epoch
source "$(dirname "$0")/gpu_round.sh"
mkdir -p gpurun_out/q
run q_ga 900 python Gradient_Averaging_main.py 3 64 1 --data_dir=synthetic:mind-small \
    --metrics_path=gpurun_out/q/ga.jsonl --snapshot_path=/tmp/q_ga.pt
run q_star 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29633 -m fedrec_with_pytorchdistributed_amd.cli star 3 1 64 --data_dir=synthetic:mind-small \
    --metrics_path=gpurun_out/q/star.jsonl --snapshot_path=/tmp/q_star.pt
