#!/bin/bash
# register-direct small GEMM vs the default form on the step's bf16 shapes (graph-timed)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r5n_rd 300 python -u benchmarks/sg_rd_bench.py gpurun_out/r5n_sg_rd.jsonl
