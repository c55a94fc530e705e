#!/bin/bash
# round-2 closing verification: smoke, the whole GPU suite, the driver's default bench,
# configs 2-5, config-2 and config-5 kernel stats
source "$(dirname "$0")/gpu_lib.sh"
check smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
check gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
run attnbench 200 python benchmarks/attn_drop_bench.py --out gpurun_out/attn_drop_bench.json
run bench_default 300 python bench.py
run c2 300 python bench.py --config 2 --steps 50 --warmup 10
run c3 300 python bench.py --config 3 --steps 50 --warmup 10
run c4 300 python bench.py --config 4 --steps 50 --warmup 10
run c5 400 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_nosplit 400 env FEDREC_TAB_DROP_SPLIT=0 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
O=$PWD/gpurun_out/prof_final_c2
rm -rf $O; mkdir -p $O
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
O=$PWD/gpurun_out/prof_final_c5
rm -rf $O; mkdir -p $O
run prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c5 -- python bench.py --config 5 --steps 4 --warmup 2 --no-valid
