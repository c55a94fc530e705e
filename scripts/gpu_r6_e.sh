#!/bin/bash
# federated quality with the server-step options (star FedAvgM / server lr; PA Adam moments + server step) at W = 4, 8
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run q_r6 1150 python -u scripts/quality_fed.py --out gpurun_out/r6_quality_fed2 --world 8 4
cat gpurun_out/r6_quality_fed2/summary.jsonl | cut -c1-300
