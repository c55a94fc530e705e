#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_th 300 $T tests/test_text_head_gpu.py -k wgrad
run hbench 200 python -u benchmarks/head_bench.py
