#!/bin/bash
# deferred split-K reduce in the head's reduce launch: tests, A/B/A/B at 50 steps, trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_af 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_deferred_reduce_gpu.py tests/test_no_library_kernels_gpu.py tests/test_text_head_gpu.py tests/test_user_step_gpu.py tests/test_small_gemm_gpu.py
run r5af_new1 200 env FEDREC_DEFER_REDUCE=1 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
run r5af_old1 200 env FEDREC_DEFER_REDUCE=0 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
run r5af_new2 200 env FEDREC_DEFER_REDUCE=1 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
run r5af_old2 200 env FEDREC_DEFER_REDUCE=0 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
O=$PWD/gpurun_out/prof_af; rm -rf $O; mkdir -p $O
run prof_af 200 rocprofv3 --kernel-trace --output-format csv -d $O -o af -- python -u bench.py --steps 10 --warmup 5 --round off --no-valid
for f in gpurun_out/r5af_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f); done
