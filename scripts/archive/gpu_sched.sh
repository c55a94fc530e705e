#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run sched 600 python benchmarks/schedule_bench.py --steps 300
