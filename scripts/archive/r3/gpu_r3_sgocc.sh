#!/bin/bash
# Small GEMM at 5 waves/SIMD (FEDREC_SG_OCC=5) vs the default: tests + config-2 bench A/B/A + kernel trace.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
FEDREC_SG_OCC=5 check sg_tests_occ5 300 $T tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py
check sg_tests 300 $T tests/test_small_gemm_gpu.py
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run bench_a 200 $B
FEDREC_SG_OCC=5 run bench_occ5 200 $B
run bench_a2 200 $B
FEDREC_SG_OCC=5 run bench_occ5b 200 $B
for f in bench_a bench_occ5 bench_a2 bench_occ5b; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
O=$PWD/gpurun_out/prof_occ5
rm -rf $O; mkdir -p $O
FEDREC_SG_OCC=5 run prof_occ5 300 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 30 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 20 --json gpurun_out/r3_c2_breakdown_occ5.json > gpurun_out/breakdown_occ5.txt 2>&1
head -16 gpurun_out/breakdown_occ5.txt
