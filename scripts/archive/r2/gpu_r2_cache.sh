#!/bin/bash
# hidden-state cache: GPU tests, cached vs re-encode bench, kernel stats of the cached step
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 600 python -u -m pytest tests/test_news_cache.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread
run bench_cache 300 python bench.py --steps 50 --warmup 10
run bench_nocache 300 python bench.py --steps 20 --warmup 5 --news-cache none --round off
O=$PWD/gpurun_out/prof_cache
mkdir -p $O
run prof_cache 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 5 --round off --no-valid
