#!/bin/bash
# wgrad stage-count A/B (4 vs 5 LDS stages), numerics at 5 stages
source "$(dirname "$0")/../../gpu_lib.sh"
FEDREC_WGRAD_NST=5 check wgtest5 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_gpu.py
FEDREC_WGRAD_NST=5 run bwd5 300 python benchmarks/bwd_gemm_bench.py --rounds 5
run bwd4 300 python benchmarks/bwd_gemm_bench.py --rounds 5
