#!/bin/bash
# interleaved next-stage loads in head_wgrad_g (and head_score2): bitwise tests, head bench, step A/B/A/B of the 4 combinations
# (ran against the tree that still had the head_wgrad_g ILV form and its setter; removed after this A/B)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_l 300 python -u -m pytest tests/test_text_head_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "row_tiles or wgrad_g"
run hb_l 200 python -u benchmarks/head_bench.py
for i in 1 2; do
  for v in 00 01 11; do
    run r6l_ilv${v}_$i 200 python -u benchmarks/ab_run.py --set head_score_set_ilv=${v:0:1} --set head_wgrad_set_ilv=${v:1:1} -- --steps 50 --warmup 10 --round off --no-valid
  done
done
grep -h "head_score\|wgrad_g" gpurun_out/hb_l.log | cut -c1-120
for f in gpurun_out/r6l_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f); done
