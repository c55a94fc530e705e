#!/bin/bash
# MFMA busy of the default ping-pong GEMM vs hipBLASLt on the QKV and FFN1 shapes (one pmc pass
# each, counters within one block's limits), and the text-head GEMM variants (timing)
source "$(dirname "$0")/gpu_lib.sh"
export TMPDIR=/tmp
for sh in qkv ffn1+gelu; do
  O=$PWD/gpurun_out/pmc_$sh
  rm -rf "$O"; mkdir -p "$O"
  run pmc_$sh 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$O" -o p1 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -- python benchmarks/gemm_bench.py --only-shape $sh --only-variants ours-pingpong-v9,lib --rounds 3
done
run gemm_model 300 python benchmarks/gemm_bench.py --rounds 7 --out gpurun_out/gemm_bench_r2.json
