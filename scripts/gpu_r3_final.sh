#!/bin/bash
# Round-3 verification of the tree: smoke, the whole GPU suite, the driver's default bench,
# configs 2-5, config-2 step breakdown (kernel trace).
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
check gputests 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
run bench_default 300 python -u bench.py
run c2 300 python -u bench.py --config 2 --steps 50 --warmup 10
run c3 300 python -u bench.py --config 3 --steps 50 --warmup 10
run c4 300 python -u bench.py --config 4 --steps 50 --warmup 10
run c5 400 python -u bench.py --config 5 --steps 10 --warmup 3 --no-valid
O=$PWD/gpurun_out/prof_final_c2
rm -rf $O; mkdir -p $O
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python -u bench.py --steps 30 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 20 --json gpurun_out/r3_c2_breakdown_final.json > gpurun_out/breakdown_final.txt 2>&1
head -30 gpurun_out/breakdown_final.txt
for f in bench_default c2 c3 c4 c5; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("steady_ms_per_step"), d.get("round_s"), d.get("round_impressions_per_s"))')"; done
