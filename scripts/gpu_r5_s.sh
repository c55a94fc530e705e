#!/bin/bash
# fused Q|K|V projection + attention forward; T tiles first in multi_cast: tests, A/B, trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_s1 600 $T tests/test_kernels_gpu.py -k "qkv_attention or multi_cast or user_attention"
check t_s2 900 $T tests/test_engine_gpu.py tests/test_step_graph.py tests/test_user_step_gpu.py tests/test_no_library_kernels_gpu.py
run r5s_new1 300 python -u bench.py --steps 50
run r5s_old1 300 env FEDREC_QKV_ATTN=0 python -u bench.py --steps 50
run r5s_new2 300 python -u bench.py --steps 50
run r5s_old2 300 env FEDREC_QKV_ATTN=0 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_r5s
rm -rf $O; mkdir -p $O
run prof_r5s 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r5_cfg2_step_breakdown_s.json > gpurun_out/breakdown_r5s.txt 2>&1
python benchmarks/launch_seq.py "$f" > gpurun_out/r5s_launch_seq.txt
for f in gpurun_out/r5s_*1.log gpurun_out/r5s_*2.log; do echo "$f $(grep -o '"steady_ms_per_step": [0-9.]*' $f)"; done
