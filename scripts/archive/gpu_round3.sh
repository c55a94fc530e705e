#!/bin/bash
# FedAvg star round at mind-small with the per-epoch schedule now using the batch lookahead
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/round
run eptests 300 python -u -m pytest tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "per_epoch or oracle"
run round_la 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29644 -m fedrec_with_pytorchdistributed_amd.cli star 2 1 64 --data_dir=synthetic:mind-small \
    --metrics_path=gpurun_out/round/star_ms_la.jsonl --snapshot_path=/tmp/rs2/s.pt
run round_la0 900 env FEDREC_LOOKAHEAD=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29645 -m fedrec_with_pytorchdistributed_amd.cli star 2 1 64 --data_dir=synthetic:mind-small \
    --metrics_path=gpurun_out/round/star_ms_la0.jsonl --snapshot_path=/tmp/rs3/s.pt
