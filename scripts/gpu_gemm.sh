#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
run kernels 900 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu
run gemm 600 python benchmarks/gemm_bench.py --out gpurun_out/gemm_bench.json
run bench 900 python bench.py --steps 10 --warmup 3
