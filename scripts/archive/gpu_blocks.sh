#!/bin/bash
# config 5 fused training blocks (residual via addmm_, GELU' in the dgrad epilogue): numerics + A/B
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run blktests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "gelu_bwd_epilogue or unfrozen or gemm_variants"
run c5_b1 400 env FEDREC_TRAIN_BLOCKS=1 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_b0 400 env FEDREC_TRAIN_BLOCKS=0 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_b1b 400 env FEDREC_TRAIN_BLOCKS=1 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
