#!/bin/bash
# round-2 verification: smoke, the GPU suite, the four BASELINE configs, a config-2 kernel profile
source "$(dirname "$0")/gpu_lib.sh"
check smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
check gputests 1100 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread
rm -f gpurun_out/configs.jsonl
for c in 2 3 4 5; do
  run bench_cfg$c 600 python bench.py --config $c --steps 50 --warmup 10
  grep -h '^{' gpurun_out/bench_cfg$c.log >> gpurun_out/configs.jsonl || true
done
O=$PWD/gpurun_out/prof_full
mkdir -p $O
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
