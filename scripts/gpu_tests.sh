#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
run gputests 1200 python -m pytest tests -q -m gpu
run smoke 600 python __graft_entry__.py smoke
run bench 900 python bench.py --steps 20 --warmup 5
