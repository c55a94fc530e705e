#!/bin/bash
# N > 1 step tails (2 clients sharing the GPU, kernel trace): the head's weight gradients written
# in place (graph run 1) vs copied at the end of the backward (graph run 2), then the eager run
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/prof_r6w; rm -rf $O; mkdir -p $O
run prof_r6w 500 rocprofv3 --kernel-trace --output-format csv -d $O -o %pid%_tr -- python -u benchmarks/early_reduce_trace.py 2
for f in $(find $O -name "*kernel_trace.csv"); do echo "== $f"; python benchmarks/step_tail.py $f --json ${f%.csv}_tail.json; done
