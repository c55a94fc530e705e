#!/bin/bash
# user pool projection inside the fused user-tail launch: tests, A/B/A/B at 50 steps, trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_ag 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -p no:cacheprovider tests/test_step_fusions_gpu.py tests/test_user_step_gpu.py tests/test_deferred_reduce_gpu.py tests/test_no_library_kernels_gpu.py tests/test_engine_gpu.py
run r5ag_new1 200 env FEDREC_POOL_E=1 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
run r5ag_old1 200 env FEDREC_POOL_E=0 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
run r5ag_new2 200 env FEDREC_POOL_E=1 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
run r5ag_old2 200 env FEDREC_POOL_E=0 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
O=$PWD/gpurun_out/prof_ag; rm -rf $O; mkdir -p $O
run prof_ag 200 rocprofv3 --kernel-trace --output-format csv -d $O -o ag -- python -u bench.py --steps 10 --warmup 5 --round off --no-valid
for f in gpurun_out/r5ag_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f); done
