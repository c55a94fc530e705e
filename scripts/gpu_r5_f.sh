#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_head 600 python -u -m pytest tests/test_text_head_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
run r5f_head_bench 300 python -u benchmarks/head_bench.py
