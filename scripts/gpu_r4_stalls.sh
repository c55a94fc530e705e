#!/bin/bash
# Wave-state counters of the closing tree's config-2 step (two --pmc passes of SQ counters,
# each its own run of the same short bench) -> benchmarks/pmc_stalls.py
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/pmc_stalls
rm -rf "$O"; mkdir -p "$O"
B="python -u bench.py --steps 20 --warmup 5 --round off --no-valid"
run pmc_s1 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC -- $B
run pmc_s2 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s2 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES -- $B
python benchmarks/pmc_stalls.py "$O" > gpurun_out/r4_pmc_stalls_cfg2.json
head -c 1500 gpurun_out/r4_pmc_stalls_cfg2.json
