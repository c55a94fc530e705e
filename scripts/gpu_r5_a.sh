#!/bin/bash
# in-graph device-epoch IPC all-reduce + cooperative cache build (shared-GPU rehearsal)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_multi 900 python -u -m pytest tests/test_multirank_gpu.py tests/test_ipc_allreduce_gpu.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider
run r5a_bench 300 python -u bench.py
