#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
run kgemm 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm"
run gemm 600 python benchmarks/gemm_bench.py --diag --out gpurun_out/gemm_bench_v10.json
