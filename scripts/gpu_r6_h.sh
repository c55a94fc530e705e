#!/bin/bash
# where the text head's X rows come from: the head kernels with the step's titles random (the real
# case), sorted, 64 distinct (cache-resident) or one title
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
for m in perm sorted pool64 same; do
  run hb_ids_$m 200 python -u benchmarks/head_bench.py --ids $m
done
for m in perm sorted pool64 same; do grep -h "head_score\"\|head_score_160\|head_pool\"\|head_pool_bwd_g\|head_wgrad_g\|head_pool_bwd\"" gpurun_out/hb_ids_$m.log | cut -c1-140; done
