#!/bin/bash
# head_score2 X-row L2 prefetch: bitwise test, standalone head bench, in-step A/B (50 steps)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_g 300 python -u -m pytest tests/test_text_head_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "row_tiles or oracle"
run hb_g 200 python -u benchmarks/head_bench.py
for i in 1 2; do
  for pf in 0 1 2; do
    run r6g_pf${pf}_$i 200 python -u benchmarks/ab_run.py --set head_score_set_pf=$pf -- --steps 50 --warmup 10 --round off --no-valid
  done
done
grep head_score gpurun_out/hb_g.log
for f in gpurun_out/r6g_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f); done
