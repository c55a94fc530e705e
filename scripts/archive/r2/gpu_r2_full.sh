#!/bin/bash
# round-2 verification: smoke, the GPU suite, the driver's default bench, the four BASELINE
# configs, a config-2 and a config-5 kernel profile
source "$(dirname "$0")/../../gpu_lib.sh"
check smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
check gputests 1100 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread
run bench_default 400 python bench.py
rm -f gpurun_out/configs.jsonl
for c in 2 3 4 5; do
  run bench_cfg$c 600 python bench.py --config $c --steps 50 --warmup 10
  grep -h '^{' gpurun_out/bench_cfg$c.log >> gpurun_out/configs.jsonl || true
done
O=$PWD/gpurun_out/prof_full
rm -rf $O; mkdir -p $O
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
run prof5 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c5 -- python bench.py --config 5 --steps 6 --warmup 3 --round off --no-valid
