#!/bin/bash
# PMC comparison: ping-pong GEMM with vs without epilogue stores (QKV shape)
source "$(dirname "$0")/gpu_round.sh"
export TMPDIR=/tmp
O=$PWD/gpurun_out/gpmc
mkdir -p $O
B="python benchmarks/gemm_bench.py --diag --only-shape qkv --only-variants ours-pingpong,diag-pingpong-nostore,lib --rounds 3"
run gp1 600 rocprofv3 --kernel-trace --output-format csv -d $O -o p1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VALU -- $B
run gp2 600 rocprofv3 --kernel-trace --output-format csv -d $O -o p2 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU -- $B
run gp3 600 rocprofv3 --kernel-trace --output-format csv -d $O -o p3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -- $B
run gp4 600 rocprofv3 --kernel-trace --output-format csv -d $O -o p4 --pmc FETCH_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum -- $B
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/q
run q_ga_lr 900 python Gradient_Averaging_main.py 4 64 1 --data_dir=synthetic:mind-small --score_act=identity --lr=1e-3 \
    --metrics_path=gpurun_out/q/ga_identity_lr1e-3.jsonl --snapshot_path=/tmp/q_ga2.pt
