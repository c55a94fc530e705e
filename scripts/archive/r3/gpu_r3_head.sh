#!/bin/bash
# Text-head variants: oracle test per head_score2 tiling, then the head microbenchmark per variant.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
for v in 1 2 3 4; do
  FEDREC_HEAD_SCORE=$v check head_oracle_s$v 200 python -u -m pytest tests/test_text_head_gpu.py -x -q --timeout 120 --timeout-method thread
done
for v in 0 1 2 3 4; do
  FEDREC_HEAD_SCORE=$v run head_bench_s$v 120 python -u benchmarks/head_bench.py --iters 30
done
FEDREC_HEAD_POOL=0 run head_bench_pool0 120 python -u benchmarks/head_bench.py --iters 30
grep -h head_ gpurun_out/head_bench_*.log > gpurun_out/head_bench_all.txt
