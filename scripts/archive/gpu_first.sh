#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
run kernels 900 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu
run smoke 600 python __graft_entry__.py smoke
run bench 900 python bench.py --steps 10 --warmup 3
