#!/bin/bash
# segment sum with the fix-up merged (one launch): tests, A/B, trace; rd small tiles; step PMC
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_w1 600 $T tests/test_kernels_gpu.py -k "segment or dedup or ldp"
check t_w2 900 $T tests/test_engine_gpu.py tests/test_step_graph.py tests/test_user_step_gpu.py
OLD="import sys, runpy; sys.argv=['bench.py','--steps','50']; from fedrec_with_pytorchdistributed_amd.ops import native; native.lib().segsum_set_variant(2); runpy.run_path('bench.py', run_name='__main__')"
run r5w_new1 300 python -u bench.py --steps 50
run r5w_old1 300 python -u -c "$OLD"
run r5w_new2 300 python -u bench.py --steps 50
run r5w_old2 300 python -u -c "$OLD"
O=$PWD/gpurun_out/prof_r5w
rm -rf $O; mkdir -p $O
run prof_r5w 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/launch_seq.py "$f" > gpurun_out/r5w_launch_seq.txt
for f in gpurun_out/r5w_*.log; do echo "$f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f|head -1)"; done
run r5v_rd 300 python -u benchmarks/sg_rd_bench.py gpurun_out/r5v_sg_rd.jsonl
