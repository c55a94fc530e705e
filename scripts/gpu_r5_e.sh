#!/bin/bash
# G path (separate g rewrite) vs round-4 head backward in the step: A/B/A/B + step breakdown
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r5e_g1 300 python -u bench.py --steps 50
run r5e_r4a 300 env FEDREC_HEAD_G=0 python -u bench.py --steps 50
run r5e_g2 300 python -u bench.py --steps 50
run r5e_r4b 300 env FEDREC_HEAD_G=0 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_r5e
rm -rf $O; mkdir -p $O
run prof_r5e 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r5_cfg2_step_breakdown_g.json > gpurun_out/breakdown_r5e.txt 2>&1
head -40 gpurun_out/breakdown_r5e.txt
