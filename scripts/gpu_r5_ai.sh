#!/bin/bash
# LDP chunk pass with the transform spread over a block per chunk: tests, config-4 A/B/A/B
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_ai 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "segment or ldp"
check t_ai2 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -p no:cacheprovider tests/test_engine_gpu.py tests/test_step_fusions_gpu.py
PRE="import sys, runpy; from fedrec_with_pytorchdistributed_amd.ops import native; native.lib().segsum_set_ldp_block"
POST="; sys.argv = ['bench.py', '--config', '4', '--steps', '50', '--warmup', '10', '--round', 'off', '--no-valid']; runpy.run_path('bench.py', run_name='__main__')"
run r5ai_new1 200 python -u -c "$PRE(1)$POST"
run r5ai_old1 200 python -u -c "$PRE(0)$POST"
run r5ai_new2 200 python -u -c "$PRE(1)$POST"
run r5ai_old2 200 python -u -c "$PRE(0)$POST"
for f in gpurun_out/r5ai_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f); done
