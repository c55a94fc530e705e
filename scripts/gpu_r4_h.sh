#!/bin/bash
# Held-batch lifetime ring instead of per-tensor record_stream (allocator event records on the
# main stream): tests, bench, step-seam profile.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_h 600 $T tests/test_step_graph.py tests/test_engine_gpu.py tests/test_multirank_gpu.py -k "graph or engine or learns or validation or two_clients"
run bench 300 python -u bench.py
O=$PWD/gpurun_out/prof_c2h
rm -rf $O; mkdir -p $O
run prof_c2h 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_h.json > gpurun_out/breakdown_c2h.txt 2>&1
head -8 gpurun_out/breakdown_c2h.txt
