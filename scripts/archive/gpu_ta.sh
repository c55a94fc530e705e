#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
export TMPDIR=/tmp
O=$PWD/gpurun_out/ta
mkdir -p $O
run kta 300 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu -k "title or engine or backbone"
run cfg2 600 python bench.py --config 2 --steps 20 --warmup 5
run prof2 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --config 2 --steps 10 --warmup 3 --no-valid
