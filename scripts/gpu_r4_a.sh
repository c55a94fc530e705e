#!/bin/bash
# Round-4 batch A: exact secure sum (histogram bound), IPC hardening + wiring, device validation.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_kern 300 $T tests/test_kernels_gpu.py -k "secagg or user_attention or score_ce"
check t_valid 300 $T tests/test_engine_gpu.py -k "validation"
check t_ipc 400 $T tests/test_ipc_allreduce_gpu.py
check t_multi 900 $T tests/test_multirank_gpu.py -k "secure or ipc"
run bench 300 python -u bench.py
run bench_c5 300 python -u bench.py --config 5 --steps 6 --warmup 3
bash scripts/gpu_r4_hosttrace.sh
