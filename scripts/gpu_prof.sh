#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p $OUT
run kernels 900 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu
run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o bench -- python bench.py --steps 10 --warmup 3 --no-valid
