#!/bin/bash
# fused user tail with x / e staged in LDS: tests, A/B, trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_aa1 600 $T tests/test_user_step_gpu.py tests/test_kernels_gpu.py -k "pool_score or score_ce or user_step"
check t_aa2 900 $T tests/test_engine_gpu.py tests/test_step_graph.py
OLD="import sys, runpy; sys.argv=['bench.py','--steps','50']; from fedrec_with_pytorchdistributed_amd.ops import native; native.lib().score_set_variant(2); runpy.run_path('bench.py', run_name='__main__')"
run r5aa_new1 300 python -u bench.py --steps 50
run r5aa_old1 300 python -u -c "$OLD"
run r5aa_new2 300 python -u bench.py --steps 50
run r5aa_old2 300 python -u -c "$OLD"
O=$PWD/gpurun_out/prof_r5aa
rm -rf $O; mkdir -p $O
run prof_r5aa 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/launch_seq.py "$f" > gpurun_out/r5aa_launch_seq.txt
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r5_cfg2_step_breakdown_aa.json > gpurun_out/breakdown_r5aa.txt 2>&1
for f in gpurun_out/r5aa_*.log; do echo "$f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f|head -1)"; done
