#!/bin/bash
# register-direct att_fc1 / dctx (W1^T cast) on the original launch structure: tests, A/B, trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_r 900 $T tests/test_engine_gpu.py tests/test_step_graph.py tests/test_user_step_gpu.py tests/test_no_library_kernels_gpu.py
run r5r_new1 300 python -u bench.py --steps 50
run r5r_old1 300 env FEDREC_SG_RD=0 python -u bench.py --steps 50
run r5r_new2 300 python -u bench.py --steps 50
run r5r_old2 300 env FEDREC_SG_RD=0 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_r5r
rm -rf $O; mkdir -p $O
run prof_r5r 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r5_cfg2_step_breakdown_r.json > gpurun_out/breakdown_r5r.txt 2>&1
python benchmarks/launch_seq.py "$f" > gpurun_out/r5r_launch_seq.txt
for f in gpurun_out/r5r_*1.log gpurun_out/r5r_*2.log; do echo "$f $(grep -o '"steady_ms_per_step": [0-9.]*' $f)"; done
