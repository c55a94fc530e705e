#!/bin/bash
# fused user attention forward at five blocks per CU: test, config-2 A/B/A/B
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_ak 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "qkv_attention or user_attention"
PRE="import sys, runpy; from fedrec_with_pytorchdistributed_amd.ops import native; native.lib().user_qkv_attn_set_five"
POST="; sys.argv = ['bench.py', '--steps', '50', '--warmup', '10', '--round', 'off', '--no-valid']; runpy.run_path('bench.py', run_name='__main__')"
run r5ak_new1 200 python -u -c "$PRE(1)$POST"
run r5ak_old1 200 python -u -c "$PRE(0)$POST"
run r5ak_new2 200 python -u -c "$PRE(1)$POST"
run r5ak_old2 200 python -u -c "$PRE(0)$POST"
O=$PWD/gpurun_out/prof_ak; rm -rf $O; mkdir -p $O
run prof_ak 200 rocprofv3 --kernel-trace --output-format csv -d $O -o ak -- python -u -c "$PRE(1); sys.argv = ['bench.py', '--steps', '10', '--warmup', '5', '--round', 'off', '--no-valid']; runpy.run_path('bench.py', run_name='__main__')"
for f in gpurun_out/r5ak_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f); done
