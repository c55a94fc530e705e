#!/bin/bash
# config 5 (unfrozen BERT-base + secure aggregation): kernel stats
source "$(dirname "$0")/gpu_round.sh"
export TMPDIR=/tmp
O=$PWD/gpurun_out/prof5
mkdir -p $O
run prof5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c5 -- python bench.py --config 5 --steps 6 --warmup 2 --no-valid
