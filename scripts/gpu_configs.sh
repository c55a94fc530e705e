#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
export TMPDIR=/tmp
O=$PWD/gpurun_out/ldp
mkdir -p $O
run cfg2 600 python bench.py --config 2 --steps 20 --warmup 5
run cfg3 600 python bench.py --config 3 --steps 20 --warmup 5
run cfg4 600 python bench.py --config 4 --steps 20 --warmup 5
run cfg5 900 python bench.py --config 5 --steps 10 --warmup 3 --valid-limit 512
run ldp1 600 rocprofv3 --kernel-trace --output-format csv -d $O -o p1 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -- python bench.py --config 4 --steps 5 --warmup 2 --no-valid
run ldp2 600 rocprofv3 --kernel-trace --output-format csv -d $O -o p2 --pmc FETCH_SIZE -- python bench.py --config 4 --steps 5 --warmup 2 --no-valid
run ldp3 600 rocprofv3 --kernel-trace --output-format csv -d $O -o p3 --pmc WRITE_SIZE TCC_HIT_sum -- python bench.py --config 4 --steps 5 --warmup 2 --no-valid
