#!/bin/bash
# ping-pong GEMM counters at K = 768 vs 3072 (same M x N): what the per-tile fixed cost is made of
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/pmc_ao; rm -rf $O; mkdir -p $O
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA"
C2="SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for K in 768 3072; do
  run pmc_ao_k${K}_a 120 timeout -s KILL 100 rocprofv3 --kernel-trace --output-format csv -d $O -o k${K}a --pmc $C1 -- python -u benchmarks/gemm_one.py --M 409600 --N 768 --K $K --variant 9 --iters 5
  run pmc_ao_k${K}_b 120 timeout -s KILL 100 rocprofv3 --kernel-trace --output-format csv -d $O -o k${K}b --pmc $C2 -- python -u benchmarks/gemm_one.py --M 409600 --N 768 --K $K --variant 9 --iters 5
done
ls $O
