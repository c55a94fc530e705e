#!/bin/bash
# dctx GEMM fused into the attention backward: tests, A/B, trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_t1 600 $T tests/test_kernels_gpu.py -k "qkv_attention or bwd_dctx or user_attention"
check t_t2 900 $T tests/test_engine_gpu.py tests/test_step_graph.py tests/test_user_step_gpu.py tests/test_no_library_kernels_gpu.py
run r5t_new1 300 python -u bench.py --steps 50
run r5t_old1 300 env FEDREC_QKV_ATTN=0 python -u bench.py --steps 50
run r5t_new2 300 python -u bench.py --steps 50
run r5t_old2 300 env FEDREC_QKV_ATTN=0 python -u bench.py --steps 50
run r5t_def 300 python -u bench.py
O=$PWD/gpurun_out/prof_r5t
rm -rf $O; mkdir -p $O
run prof_r5t 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r5_cfg2_step_breakdown_t.json > gpurun_out/breakdown_r5t.txt 2>&1
python benchmarks/launch_seq.py "$f" > gpurun_out/r5t_launch_seq.txt
for f in gpurun_out/r5t_*.log; do echo "$f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f|head -1)"; done
