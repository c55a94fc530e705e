#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
export TMPDIR=/tmp
O=$PWD/gpurun_out/pmc
mkdir -p $O
run pmc1 600 rocprofv3 --kernel-trace --output-format csv -d $O -o v2a --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -- python benchmarks/gemm_one.py --variant 2
run pmc2 600 rocprofv3 --kernel-trace --output-format csv -d $O -o v2b --pmc TCC_HIT_sum TCC_MISS_sum -- python benchmarks/gemm_one.py --variant 2
run pmc3 600 rocprofv3 --kernel-trace --output-format csv -d $O -o lib --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -- python benchmarks/gemm_one.py --lib
run pmc4 600 rocprofv3 --kernel-trace --output-format csv -d $O -o libb --pmc TCC_HIT_sum TCC_MISS_sum -- python benchmarks/gemm_one.py --lib
