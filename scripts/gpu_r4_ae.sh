#!/bin/bash
# probe: the text fc backward launch, mixed dtypes vs bf16 hi/lo operands on the DMA ring
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run probe 200 python -u benchmarks/sg_mixed_probe.py gpurun_out/r4_sg_mixed_probe.json
