#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
run gemmsq 600 python benchmarks/gemm_bench.py --shapes square --rounds 5 --out gpurun_out/gemm_bench_sq.json
