#!/bin/bash
# The step-graph seam: back-to-back replays of the real step graph (events + kernel trace).
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run seam 200 python -u benchmarks/graph_seam.py --replays 40
O=$PWD/gpurun_out/prof_gseam
rm -rf $O; mkdir -p $O
run prof_gseam 300 rocprofv3 --kernel-trace --output-format csv -d $O -o g -- python -u benchmarks/graph_seam.py --replays 20
ls $O
