#!/bin/bash
# (run while the two buffers were opt-in; they are the default now, FEDREC_SG_DB=0 = one buffer)
# Small GEMM with two LDS buffers and one barrier per k-step (FEDREC_SG_DB=1) vs the default:
# numerics under the switch, then bench arms A/B/A/B.
source "$(dirname "$0")/../../gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
FEDREC_SG_DB=1 check t_db 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run b_def 200 $B
FEDREC_SG_DB=1 run b_db 200 $B
run b_def2 200 $B
FEDREC_SG_DB=1 run b_db2 200 $B
run b_def3 200 $B
FEDREC_SG_DB=1 run b_db3 200 $B
for f in b_def b_db b_def2 b_db2 b_def3 b_db3; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
O=$PWD/gpurun_out/prof_db
rm -rf $O; mkdir -p $O
FEDREC_SG_DB=1 run prof_db 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o db -- python -u bench.py --steps 30 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 20 > gpurun_out/breakdown_db.txt 2>&1
head -14 gpurun_out/breakdown_db.txt
