#!/bin/bash
# Small-GEMM split-K granularity: fewest K per split (FEDREC_SG_MINK, arms via MINKS) vs 384 (default):
# small-GEMM tests under the switch, bench arms, and the kernel breakdown of the 256 arm.
source "$(dirname "$0")/../../gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
FEDREC_SG_MINK=192 check t_mink 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
MINKS=${MINKS:-"256 192"}
names=""
for r in 1 2; do
  run b_def$r 200 $B; names="$names b_def$r"
  for m in $MINKS; do FEDREC_SG_MINK=$m run b_${m}_$r 200 $B; names="$names b_${m}_$r"; done
done
for f in $names; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
