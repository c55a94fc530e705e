#!/bin/bash
# config 4 on the captured step (LDP noise offset from the device step counter), int32 gathers:
# targeted tests, config 4 / config 2 benches, config-4 graph on/off A/B
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_step_graph.py tests/test_engine_gpu.py tests/test_user_step_gpu.py tests/test_multirank_gpu.py tests/test_kernels_gpu.py
run c4_graph 300 python bench.py --config 4 --steps 50 --warmup 10
run c4_eager 300 env FEDREC_STEP_GRAPH=off python bench.py --config 4 --steps 50 --warmup 10
run c2 300 python bench.py --steps 50 --warmup 10
run c2_default 300 python bench.py
