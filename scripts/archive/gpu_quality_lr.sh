#!/bin/bash
# Training-quality runs on the planted-signal synthetic shard (mind-small, 1 client, GA, B=64).
#  * the reference model exactly (sigmoid-CE scorer, lr 5e-5)
#  * plain-CE scorer at lr 1e-4 / 1e-3 (random-init heads; 5e-5 is tuned for pretrained BERT)
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/q
E=${EPOCHS:-3}
run q_sig_lr5e-5 600 python Gradient_Averaging_main.py $E 64 1 --data_dir=synthetic:mind-small \
    --metrics_path=gpurun_out/q/ga_sigmoid_lr5e-5.jsonl --snapshot_path=/tmp/q0.pt
run q_id_lr1e-4 600 python Gradient_Averaging_main.py $E 64 1 --data_dir=synthetic:mind-small --lr=1e-4 --score_act=identity \
    --metrics_path=gpurun_out/q/ga_identity_lr1e-4.jsonl --snapshot_path=/tmp/q1.pt
run q_id_lr1e-3 600 python Gradient_Averaging_main.py $E 64 1 --data_dir=synthetic:mind-small --lr=1e-3 --score_act=identity \
    --metrics_path=gpurun_out/q/ga_identity_lr1e-3.jsonl --snapshot_path=/tmp/q2.pt
