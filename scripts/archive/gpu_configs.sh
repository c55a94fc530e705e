#!/bin/bash
# GPU tests, then the four BASELINE configs on one GPU (bench.py JSON lines -> gpurun_out/configs.jsonl)
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
for c in 2 3 4 5; do
  run bench_cfg$c 600 python bench.py --config $c --steps 30 --warmup 5
  grep '^{' gpurun_out/bench_cfg$c.log >> gpurun_out/configs.jsonl
done
