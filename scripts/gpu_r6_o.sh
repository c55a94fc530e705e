#!/bin/bash
# adam_dev with the first element's p / m / v loads ahead of the table + bias corrections:
# kernel test, step A/B/A/B, then a kernel-trace breakdown of the (prefetching) step
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_o 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "adam or graph"
for i in 1 2; do
  for v in 0 1; do
    run r6o_pf${v}_$i 200 python -u benchmarks/ab_run.py --set adam_dev_set_prefetch=$v -- --steps 50 --warmup 10 --round off --no-valid
  done
done
O=$PWD/gpurun_out/prof_r6o; rm -rf $O; mkdir -p $O
run prof_r6o 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o ar -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
python benchmarks/launch_seq.py $O/ar_kernel_trace.csv > gpurun_out/r6_cfg2_launch_seq_o.txt 2>&1
python benchmarks/step_breakdown.py $O/ar_kernel_trace.csv --steps 10 --json gpurun_out/r6_cfg2_step_breakdown_o.json > gpurun_out/r6_breakdown_o.txt 2>&1
head -24 gpurun_out/r6_breakdown_o.txt
for f in gpurun_out/r6o_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f); done
