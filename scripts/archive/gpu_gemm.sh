#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
run kgemm 900 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm"
run gemm 600 python benchmarks/gemm_bench.py --out gpurun_out/gemm_bench.json
