#!/bin/bash
# step graphs: equivalence test, cached bench with graphs on/off, kernel trace
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 600 python -u -m pytest tests/test_step_graph.py tests/test_news_cache.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread
run bench_graph 300 python bench.py --steps 50 --warmup 10
run bench_nograph 300 env FEDREC_STEP_GRAPH=off python bench.py --steps 50 --warmup 10 --round off
O=$PWD/gpurun_out/prof_graph
mkdir -p $O
run prof_graph 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
