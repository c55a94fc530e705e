#!/bin/bash
# FedAvg round wall-clock at the reference's measured scale (1 server +
# clients, batch 2, 1 local epoch over the shipped-shard-sized data -> 14.6-15.2 s/round on
# CPU): coordinator (rank 0, CPU) + 1 MI355X client, toy preset (1 user, 4 + 1 impressions,
# 224 news), 5 rounds; and the same at mind-small scale (one full local epoch per round).
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/round
run round_toy 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29641 -m fedrec_with_pytorchdistributed_amd.cli star 5 1 2 --data_dir=synthetic:toy \
    --metrics_path=gpurun_out/round/star_toy.jsonl --snapshot_path=/tmp/rt/s.pt
run round_small 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29642 -m fedrec_with_pytorchdistributed_amd.cli star 2 1 64 --data_dir=synthetic:mind-small \
    --metrics_path=gpurun_out/round/star_mind_small.jsonl --snapshot_path=/tmp/rs/s.pt
