#!/bin/bash
# segment sum with the edge fix-up inside the chunk launch: kernel tests (bitwise vs two launches),
# engine tests, step A/B/A/B (config 2 and config 4 = LDP), kernel trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_s 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "segment or dedup or ldp"
check t_s2 600 python -u -m pytest tests/test_engine_gpu.py tests/test_step_fusions_gpu.py tests/test_step_graph.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for i in 1 2; do
  for v in 0 1; do
    run r6s_fx${v}_$i 200 python -u benchmarks/ab_run.py --set segsum_set_fused_fix=$v -- --steps 50 --warmup 10 --round off --no-valid
  done
done
for v in 0 1; do
  run r6s_c4_fx${v} 200 python -u benchmarks/ab_run.py --set segsum_set_fused_fix=$v -- --config 4 --steps 50 --warmup 10 --round off --no-valid
done
O=$PWD/gpurun_out/prof_r6s; rm -rf $O; mkdir -p $O
run prof_r6s 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o ar -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
python benchmarks/launch_seq.py $O/ar_kernel_trace.csv > gpurun_out/r6_cfg2_launch_seq_s.txt 2>&1
python benchmarks/step_breakdown.py $O/ar_kernel_trace.csv --steps 10 --json gpurun_out/r6_cfg2_step_breakdown_s.json > gpurun_out/r6_breakdown_s.txt 2>&1
head -24 gpurun_out/r6_breakdown_s.txt
for f in gpurun_out/r6s_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f); done
