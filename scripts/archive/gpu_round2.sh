#!/bin/bash
# Full check after a kernel change: GPU tests, configs 2-5, a rocprofv3 kernel-stats profile of config 2.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
rm -f gpurun_out/configs.jsonl
run gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
for c in 2 3 4 5; do
  run bench_cfg$c 600 python bench.py --config $c --steps 30 --warmup 5
  grep '^{' gpurun_out/bench_cfg$c.log >> gpurun_out/configs.jsonl
done
mkdir -p gpurun_out/prof
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/prof -o bench -- python bench.py --steps 10 --warmup 3 --no-valid
