#!/bin/bash
# config-5 glue: one-launch compute-weight refresh, LN2 backward with the FFN dropout backward
# fused, dropout-case QKV bias shortcut, no fp32 q|k|v cat; full GPU suite + config-5 A/B
source "$(dirname "$0")/../../gpu_lib.sh"
check gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
run c5_a 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_nofuse 400 env FEDREC_LN_DROP_FUSE=0 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_b 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
O=$PWD/gpurun_out/prof_c5
rm -rf $O; mkdir -p $O
run prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c5 -- python bench.py --config 5 --steps 4 --warmup 2 --no-valid
