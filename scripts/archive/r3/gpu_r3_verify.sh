#!/bin/bash
# Re-entry verification: smoke, the whole GPU suite, the default bench, a kernel-trace step breakdown.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
bash scripts/gpu_r3_head.sh || exit 1
check gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench 300 python -u bench.py
run prof 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c2 -o c2 -- python -u bench.py --steps 30 --warmup 5 --round off --no-valid
f=$(find gpurun_out/prof_c2 -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 20 --json gpurun_out/r3_c2_breakdown.json > gpurun_out/breakdown.txt 2>&1
head -40 gpurun_out/breakdown.txt
bash scripts/gpu_r3_stepmc.sh
