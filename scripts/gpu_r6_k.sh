#!/bin/bash
# head_score2 with the next stage's loads interleaved with the MFMA rows: bitwise test, head bench, step A/B
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_k 300 python -u -m pytest tests/test_text_head_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "row_tiles"
run hb_k 200 python -u benchmarks/head_bench.py
for i in 1 2; do
  for v in 0 1; do
    run r6k_ilv${v}_$i 200 python -u benchmarks/ab_run.py --set head_score_set_ilv=$v -- --steps 50 --warmup 10 --round off --no-valid
  done
done
grep -h "head_score" gpurun_out/hb_k.log | cut -c1-120
for f in gpurun_out/r6k_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f); done
