#!/bin/bash
# the step's input launch (multi_cast) with one load -> store round trip per block (iters 1)
# vs the round-5 form (4 serialised iterations): tests, step A/B/A/B, kernel trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_q 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_step_graph.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "cast or graph or adam or flat"
for i in 1 2; do
  for v in 4 1; do
    run r6q_it${v}_$i 200 python -u benchmarks/ab_run.py --set multi_cast_set_iters=$v -- --steps 50 --warmup 10 --round off --no-valid
  done
done
O=$PWD/gpurun_out/prof_r6q; rm -rf $O; mkdir -p $O
run prof_r6q 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o ar -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
python benchmarks/launch_seq.py $O/ar_kernel_trace.csv > gpurun_out/r6_cfg2_launch_seq_q.txt 2>&1
python benchmarks/step_breakdown.py $O/ar_kernel_trace.csv --steps 10 --json gpurun_out/r6_cfg2_step_breakdown_q.json > gpurun_out/r6_breakdown_q.txt 2>&1
head -24 gpurun_out/r6_breakdown_q.txt
for f in gpurun_out/r6q_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f); done
