#!/bin/bash
# round-2 re-entry check: smoke, the GPU suite, default bench, config-2 kernel stats
source "$(dirname "$0")/gpu_lib.sh"
check smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
check gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
run bench_default 300 python bench.py
O=$PWD/gpurun_out/prof2
mkdir -p $O
run prof2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 10 --warmup 3 --no-valid
