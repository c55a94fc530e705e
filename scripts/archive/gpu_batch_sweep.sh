#!/bin/bash
# Config 2 at several per-GPU batch sizes (bench default: 64), then configs 3-5.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
rm -f gpurun_out/sweep.jsonl gpurun_out/configs.jsonl
for b in 16 32 64 128 256; do
  run bench_b$b 300 python bench.py --batch $b --steps 20 --warmup 5 --no-valid
  grep '^{' gpurun_out/bench_b$b.log >> gpurun_out/sweep.jsonl
done
for c in 2 3 4 5; do
  run bench_cfg$c 600 python bench.py --config $c --steps 30 --warmup 5
  grep '^{' gpurun_out/bench_cfg$c.log >> gpurun_out/configs.jsonl
done
