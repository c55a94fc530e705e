#!/bin/bash
# head_score2 160-row tile: tests, head bench A/B, bench.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_t 600 $T tests/test_text_head_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py
run hbench 200 python -u benchmarks/head_bench.py --U 1600
run bench 300 python -u bench.py
run bench50 300 python -u bench.py --steps 50
