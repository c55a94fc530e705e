#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
run gputests 1200 python -m pytest tests -x -q -m gpu
run bench 900 python bench.py --steps 10 --warmup 3
