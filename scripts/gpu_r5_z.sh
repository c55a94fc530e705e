#!/bin/bash
# side-stream weight gradients vs hardware-queue count (the lookahead stream behind a graph branch?)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r5z_def1 300 python -u bench.py --steps 50
run r5z_side1 300 env FEDREC_SIDE_WGRAD=1 python -u bench.py --steps 50
run r5z_sideq1 300 env FEDREC_SIDE_WGRAD=1 GPU_MAX_HW_QUEUES=8 python -u bench.py --steps 50
run r5z_defq1 300 env GPU_MAX_HW_QUEUES=8 python -u bench.py --steps 50
run r5z_def2 300 python -u bench.py --steps 50
run r5z_sideq2 300 env FEDREC_SIDE_WGRAD=1 GPU_MAX_HW_QUEUES=8 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_r5z
rm -rf $O; mkdir -p $O
export FEDREC_SIDE_WGRAD=1 GPU_MAX_HW_QUEUES=8
run prof_r5z 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/launch_seq.py "$f" > gpurun_out/r5z_launch_seq.txt
for f in gpurun_out/r5z_*.log; do echo "$f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"next_batch": [0-9.]*' $f)"; done
