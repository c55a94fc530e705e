#!/bin/bash
# HIP API + kernel trace of the config-2 bench: where the host is when the GPU idles between steps.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/prof_ht
rm -rf $O; mkdir -p $O
run prof_ht 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O -o ht -- python -u bench.py --steps 12 --warmup 5 --round off --no-valid
ls -la $O
