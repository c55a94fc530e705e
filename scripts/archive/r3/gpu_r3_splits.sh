#!/bin/bash
# head_wgrad split count in the step: default (CUs - 16) / 9 = 26 vs 28 (all CUs: the lookahead
# stream's dedup has finished by the time the weight gradient runs) vs 27.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run b_def 200 $B
FEDREC_HEAD_SPLITS=28 run b_s28 200 $B
FEDREC_HEAD_SPLITS=27 run b_s27 200 $B
run b_def2 200 $B
FEDREC_HEAD_SPLITS=28 run b_s28b 200 $B
for f in b_def b_s28 b_s27 b_def2 b_s28b; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
