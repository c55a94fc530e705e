#!/bin/bash
# full GPU suite, the four BASELINE configs, and a config-2 kernel profile
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
rm -f gpurun_out/configs.jsonl
for c in 2 3 4 5; do
  run bench_cfg$c 600 python bench.py --config $c --steps 30 --warmup 5
  grep -h '^{' gpurun_out/bench_cfg$c.log >> gpurun_out/configs.jsonl || true
done
O=$PWD/gpurun_out/prof2
mkdir -p $O
run prof2 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --config 2 --steps 10 --warmup 3 --no-valid
