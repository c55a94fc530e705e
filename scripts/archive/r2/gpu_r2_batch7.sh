#!/bin/bash
# wgrad LDS stage count for config 5 (3 = default, chosen for config 2's one-wave head wgrad)
# and refreshed configs 3 / 4 numbers
source "$(dirname "$0")/../../gpu_lib.sh"
run c5_nst3 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_nst4 400 env FEDREC_WGRAD_NST=4 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_nst3b 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_nst4b 400 env FEDREC_WGRAD_NST=4 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c3 300 python bench.py --config 3 --steps 50 --warmup 10
run c4 300 python bench.py --config 4 --steps 50 --warmup 10
