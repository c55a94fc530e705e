#!/bin/bash
# Small GEMM with stored-transposed operands staged as TRI images (default; FEDREC_SG_TR=0 = the
# scalar-transposed-store image): numerics (small-GEMM, user-step, step-graph, text-head tests),
# then bench arms A/B/A/B.  Recorded in profiles/r3_ab_sg_tri.txt (run while TRI was opt-in).
source "$(dirname "$0")/../../gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_tr 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py tests/test_step_graph.py tests/test_text_head_gpu.py
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
FEDREC_SG_TR=0 run b_def 200 $B
run b_tr 200 $B
FEDREC_SG_TR=0 run b_def2 200 $B
run b_tr2 200 $B
for f in b_def b_tr b_def2 b_tr2; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
