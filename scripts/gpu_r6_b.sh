#!/bin/bash
# fused score + pool (v2: full titles first, 3 items per pass): text-head GPU tests, A/B/A/B, kernel trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_head 600 python -u -m pytest tests/test_text_head_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
for i in 1 2; do
  run r6b_fused_$i 200 python -u benchmarks/ab_run.py -- --steps 50 --warmup 10 --round off --no-valid
  run r6b_two_$i 200 python -u benchmarks/ab_run.py --set head_score_pool_set=0 -- --steps 50 --warmup 10 --round off --no-valid
done
O=$PWD/gpurun_out/prof_r6b; rm -rf $O; mkdir -p $O
run prof_r6b 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o ar -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
python benchmarks/step_breakdown.py $O/ar_kernel_trace.csv --steps 10 --json gpurun_out/r6_cfg2_step_breakdown_b.json > gpurun_out/r6_breakdown_b.txt 2>&1
head -24 gpurun_out/r6_breakdown_b.txt
for f in gpurun_out/r6b_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f); done
