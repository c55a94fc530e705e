#!/bin/bash
# TN wgrad kernel: numerics tests, then the backward-GEMM microbench
source "$(dirname "$0")/../../gpu_lib.sh"
check wgtest 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wgrad_gpu.py
run bwdgemm 300 python benchmarks/bwd_gemm_bench.py
