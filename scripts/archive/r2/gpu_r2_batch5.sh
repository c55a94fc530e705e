#!/bin/bash
# after dropping the keep-bits attention path and the ILP user-attention backward: GPU suite,
# config-2 / config-5 benches (A/B of the fused LN2 + FFN-dropout backward), config-2 profile
source "$(dirname "$0")/../../gpu_lib.sh"
check gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
run uabench 200 python benchmarks/user_attn_bench.py --out gpurun_out/user_attn_bench.json
run c2_a 300 python bench.py --steps 50 --warmup 10
run c2_default 300 python bench.py
run c5_a 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_nofuse 400 env FEDREC_LN_DROP_FUSE=0 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_b 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
O=$PWD/gpurun_out/prof_c2
rm -rf $O; mkdir -p $O
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
