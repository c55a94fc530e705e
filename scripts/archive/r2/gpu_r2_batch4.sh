#!/bin/bash
# config-5 glue (one-launch weight refresh, LN2 bwd + FFN dropout bwd, bias shortcut, no fp32
# q|k|v cat, stored attention keep bits) + config-2 (ILP user attention, split-K dgrad with the
# dropout epilogue): full GPU suite, micro A/Bs, bench A/Bs, profiles
source "$(dirname "$0")/../../gpu_lib.sh"
check gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
run attnbench 200 python benchmarks/attn_drop_bench.py --out gpurun_out/attn_drop_bench.json
run uabench 200 python benchmarks/user_attn_bench.py --out gpurun_out/user_attn_bench.json
run c2_a 300 python bench.py --steps 50 --warmup 10
run c2_ua0 300 env FEDREC_UA_VARIANT=0 python bench.py --steps 50 --warmup 10
run c2_b 300 python bench.py --steps 50 --warmup 10
run c5_a 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_old 400 env FEDREC_LN_DROP_FUSE=0 FEDREC_ATTN_BITS=0 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_b 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
O=$PWD/gpurun_out/prof_c5
rm -rf $O; mkdir -p $O
run prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c5 -- python bench.py --config 5 --steps 4 --warmup 2 --no-valid
O=$PWD/gpurun_out/prof_c2
rm -rf $O; mkdir -p $O
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
