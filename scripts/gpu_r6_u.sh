#!/bin/bash
# head_score2 with 32-wide k-tiles and 4 LDS stages (three in flight) vs 64 x 2: bitwise test,
# standalone bench, step A/B/A/B
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_u 300 python -u -m pytest tests/test_text_head_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run hb_u 200 python -u benchmarks/head_bench.py
for i in 1 2; do
  for v in 64 32; do
    run r6u_bk${v}_$i 200 python -u benchmarks/ab_run.py --set head_score_set_bk=$v -- --steps 50 --warmup 10 --round off --no-valid
  done
done
grep -h "head_score" gpurun_out/hb_u.log | cut -c1-110
for f in gpurun_out/r6u_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f); done
