#!/bin/bash
# rd small-tile variants (graph-timed) + the step's PMC passes
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r5v_rd 300 python -u benchmarks/sg_rd_bench.py gpurun_out/r5v_sg_rd.jsonl
bash scripts/gpu_r5_u.sh
