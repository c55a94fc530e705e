#!/bin/bash
# persistent title-attention backward (config 5): numerics, kernel A/B, config-5 step A/B
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run tabtests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "title_attention_bwd or unfrozen"
run tabk1 200 env FEDREC_TAB_VARIANT=1 python benchmarks/kernel_bench.py --only title_attention_bwd
run tabk0 200 env FEDREC_TAB_VARIANT=0 python benchmarks/kernel_bench.py --only title_attention_bwd
run c5_v1 400 env FEDREC_TAB_VARIANT=1 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_v0 400 env FEDREC_TAB_VARIANT=0 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
