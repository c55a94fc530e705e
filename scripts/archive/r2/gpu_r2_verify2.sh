#!/bin/bash
# multi_cast for any size / alignment, flat-gradient gather by multi_cast: GPU suite + benches
source "$(dirname "$0")/../../gpu_lib.sh"
check gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
run c2 300 python bench.py --steps 50 --warmup 10
run c2_default 300 python bench.py
run c5 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c4 300 python bench.py --config 4 --steps 50 --warmup 10
