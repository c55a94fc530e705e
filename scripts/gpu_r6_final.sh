#!/bin/bash
# round-6 closing call on the committed tree: full GPU suite + smoke, configs 2 (driver default
# and 50 steps) / 3 / 4 / 5, and the config-2 kernel-trace breakdown
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_final 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
check smoke_final 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run final_c2 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
run final_c2_50 200 python -u bench.py --gpus 1 --steps 50 --warmup 10 --no-probe
run final_c3 200 python -u bench.py --config 3
run final_c4 200 python -u bench.py --config 4
run final_c5 400 python -u bench.py --config 5
O=$PWD/gpurun_out/prof_final; rm -rf $O; mkdir -p $O
run prof_final 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o ar -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
python benchmarks/launch_seq.py $O/ar_kernel_trace.csv > gpurun_out/r6_cfg2_launch_seq_final.txt 2>&1
python benchmarks/step_breakdown.py $O/ar_kernel_trace.csv --steps 10 --json gpurun_out/r6_cfg2_step_breakdown_final.json > gpurun_out/r6_breakdown_final.txt 2>&1
cp $O/ar_kernel_stats.csv gpurun_out/r6_final_kernel_stats.csv
tail -3 gpurun_out/t_final.log
grep -h -o '"value": [0-9.]*\|"steady_ms_per_step": [0-9.]*\|"baseline_config": [0-9]\|"cache_build_ms": [0-9.]*' gpurun_out/final_c*.log
head -22 gpurun_out/r6_breakdown_final.txt
