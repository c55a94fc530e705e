#!/bin/bash
# identity-scorer collapse: where the eps-softmax cliff is crossed (1 epoch, lr 1e-3)
source "$(dirname "$0")/../../gpu_lib.sh"
run q_id_1e3b 300 python benchmarks/quality_diag.py --lr 1e-3 --score-act identity --epochs 1 --out gpurun_out/quality_identity_lr1e-3_cliff.jsonl
