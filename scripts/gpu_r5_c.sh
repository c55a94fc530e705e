#!/bin/bash
# text head G path: numerics + kernel timings + bench A/B
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_head 600 python -u -m pytest tests/test_text_head_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
run r5c_head_bench 300 python -u benchmarks/head_bench.py
run r5c_bench_g 300 python -u bench.py --steps 50
run r5c_bench_r4 300 env FEDREC_HEAD_G=0 python -u bench.py --steps 50
run r5c_bench_g2 300 python -u bench.py --steps 50
