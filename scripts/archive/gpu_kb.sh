#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
run kta 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "title or layer_norm or embed_ln or additive or wgrad"
run kb 300 python benchmarks/kernel_bench.py --out gpurun_out/kernel_bench.json
