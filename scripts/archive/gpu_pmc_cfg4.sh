#!/bin/bash
# PMC passes over a short config-4 (LDP) bench (one counter group per run; kernel trace only)
source "$(dirname "$0")/gpu_round.sh"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$PWD/gpurun_out/pmc4
mkdir -p $O
B="python bench.py --config 4 --steps 3 --warmup 2 --no-valid"
run pm1 300 rocprofv3 --kernel-trace --output-format csv -d $O -o p1 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -- $B
run pm2 300 rocprofv3 --kernel-trace --output-format csv -d $O -o p2 --pmc FETCH_SIZE -- $B
run pm3 300 rocprofv3 --kernel-trace --output-format csv -d $O -o p3 --pmc WRITE_SIZE SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU -- $B
run prof4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o s4 -- python bench.py --config 4 --steps 10 --warmup 3 --no-valid
python benchmarks/pmc_summary.py $O > gpurun_out/pmc_r1_cfg4.json
