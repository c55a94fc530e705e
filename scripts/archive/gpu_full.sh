#!/bin/bash
# tests + GEMM bench + config 2/4 bench + profile (the standard measure step)
source "$(dirname "$0")/gpu_round.sh"
export TMPDIR=/tmp
O=$PWD/gpurun_out/full
mkdir -p $O
run gputests 1200 python -m pytest tests -q -m gpu -x
run gemm 600 python benchmarks/gemm_bench.py --diag --out gpurun_out/gemm_bench_full.json
run cfg2 600 python bench.py --config 2 --steps 20 --warmup 5
run cfg4 600 python bench.py --config 4 --steps 20 --warmup 5
run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --config 2 --steps 10 --warmup 3 --no-valid
