#!/bin/bash
# config-5 backward GEMMs: microbench (ours-NT-on-W^T vs hipBLASLt) + a config-5 kernel profile
source "$(dirname "$0")/../../gpu_lib.sh"
run bwdgemm 300 python benchmarks/bwd_gemm_bench.py
O=$PWD/gpurun_out/prof_c5
mkdir -p $O
run prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c5 -- python bench.py --config 5 --steps 6 --warmup 3 --round off --no-valid
