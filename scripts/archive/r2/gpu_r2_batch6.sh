#!/bin/bash
# split step graph (hidden-row gather ahead of the optimizer wait) and the transposed bf16
# weight copies of the unfrozen backbone: targeted tests, then A/B/A benches
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py tests/test_dropout.py tests/test_user_step_gpu.py tests/test_multirank_gpu.py
run c2_a 300 python bench.py --steps 50 --warmup 10
run c2_nosplit 300 env FEDREC_SPLIT_GRAPH=0 python bench.py --steps 50 --warmup 10
run c2_b 300 python bench.py --steps 50 --warmup 10
run c5_a 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_nowt 400 env FEDREC_WT_CACHE=0 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_b 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
