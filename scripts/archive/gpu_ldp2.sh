#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
export TMPDIR=/tmp
O=$PWD/gpurun_out/ldp2
mkdir -p $O
run gputests 1200 python -m pytest tests -q -m gpu -x
run cfg2 600 python bench.py --config 2 --steps 20 --warmup 5
run cfg4 600 python bench.py --config 4 --steps 20 --warmup 5
run prof4 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c4 -- python bench.py --config 4 --steps 10 --warmup 3 --no-valid
