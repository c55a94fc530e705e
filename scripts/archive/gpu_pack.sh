#!/bin/bash
# Packed title rows: new kernel tests, the full GPU suite, then config 2 with packing on / off.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run packtests 300 python -u -m pytest tests/test_packed_gpu.py -x -v --timeout 120 --timeout-method thread
run gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
run bench_pack 300 python bench.py --steps 30 --warmup 5
FEDREC_TITLE_PACK=0 run bench_nopack 300 python bench.py --steps 30 --warmup 5
run bench_pack2 300 python bench.py --steps 30 --warmup 5
