#!/bin/bash
# ping-pong GEMM: per-tile fixed cost (K sweep at M = 409,600)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r5am_ksweep 400 python -u benchmarks/gemm_k_sweep.py gpurun_out/r5_gemm_k_sweep.jsonl
cat gpurun_out/r5am_ksweep.log
