#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p $OUT
run bench 900 python bench.py --steps 20 --warmup 5
run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o bench -- python bench.py --steps 10 --warmup 3 --no-valid
