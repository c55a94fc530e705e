#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
run kln 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "layer_norm or embed_ln"
run kb 300 python benchmarks/kernel_bench.py --only layer_norm --out gpurun_out/kernel_bench_ln.json
run gemm 600 python benchmarks/gemm_bench.py --shapes nores --out gpurun_out/gemm_bench_nores.json
