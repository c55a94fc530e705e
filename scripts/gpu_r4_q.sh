#!/bin/bash
# full GPU suite + smoke, bench (default / 50 steps), config-5 bench, step profile.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_all 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
check smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 300 python -u bench.py
run bench50 300 python -u bench.py --steps 50
run bench_c5 400 python -u bench.py --config 5 --steps 6 --warmup 3
O=$PWD/gpurun_out/prof_c2q
rm -rf $O; mkdir -p $O
run prof_c2q 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_q.json > gpurun_out/breakdown_c2q.txt 2>&1
head -32 gpurun_out/breakdown_c2q.txt
