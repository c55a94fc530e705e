#!/bin/bash
# Small-GEMM register queue depth on the TRI kernels: FEDREC_SG_NQ=2 (two k-tiles in flight,
# 2-3 waves per SIMD) and =3 (two only for launches of <= 512 tiles) vs the default one.
source "$(dirname "$0")/../../gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
FEDREC_SG_NQ=2 check t_nq 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run b_def 200 $B
FEDREC_SG_NQ=2 run b_nq2 200 $B
FEDREC_SG_NQ=3 run b_nq3 200 $B
run b_def2 200 $B
FEDREC_SG_NQ=2 run b_nq2b 200 $B
FEDREC_SG_NQ=3 run b_nq3b 200 $B
for f in b_def b_nq2 b_nq3 b_def2 b_nq2b b_nq3b; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
O=$PWD/gpurun_out/prof_nq2
rm -rf $O; mkdir -p $O
FEDREC_SG_NQ=2 run prof_nq2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o nq2 -- python -u bench.py --steps 30 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 20 > gpurun_out/breakdown_nq2.txt 2>&1
head -16 gpurun_out/breakdown_nq2.txt
