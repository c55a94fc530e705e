#!/bin/bash
# persistent dropout attention fwd/bwd: micro A/B, dropout + backbone tests, config-5 A/B
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dropout.py tests/test_kernels_gpu.py -m gpu tests/test_engine_gpu.py -k "attention or dropout or unfrozen"
run attnbench 200 python benchmarks/attn_drop_bench.py --out gpurun_out/attn_drop_bench.json
run c5_new 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_old 400 env FEDREC_TAB_VARIANT=0 FEDREC_TA_WAVES=2 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_new2 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
