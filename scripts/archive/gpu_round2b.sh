#!/bin/bash
# FedAvg star round wall-clock at mind-small (coordinator + 1 MI355X client): validation with a
# per-pass news table (default) vs per-batch encoding, plus the new test
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/round
run vtest 300 python -u -m pytest tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "validation_news_table"
run round_t1 900 env FEDREC_VALID_TABLE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29642 -m fedrec_with_pytorchdistributed_amd.cli star 2 1 64 --data_dir=synthetic:mind-small \
    --metrics_path=gpurun_out/round/star_ms_t1.jsonl --snapshot_path=/tmp/rs1/s.pt
run round_t0 900 env FEDREC_VALID_TABLE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29643 -m fedrec_with_pytorchdistributed_amd.cli star 2 1 64 --data_dir=synthetic:mind-small \
    --metrics_path=gpurun_out/round/star_ms_t0.jsonl --snapshot_path=/tmp/rs0/s.pt
