#!/bin/bash
# plain segment sum on a block per chunk: test, config-2 A/B/A/B
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_aj 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "segment or ldp"
PRE="import sys, runpy; from fedrec_with_pytorchdistributed_amd.ops import native; native.lib().segsum_set_ldp_block"
POST="; sys.argv = ['bench.py', '--steps', '50', '--warmup', '10', '--round', 'off', '--no-valid']; runpy.run_path('bench.py', run_name='__main__')"
run r5aj_new1 200 python -u -c "$PRE(3)$POST"
run r5aj_old1 200 python -u -c "$PRE(1)$POST"
run r5aj_new2 200 python -u -c "$PRE(3)$POST"
run r5aj_old2 200 python -u -c "$PRE(1)$POST"
for f in gpurun_out/r5aj_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f); done
