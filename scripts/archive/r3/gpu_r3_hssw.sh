#!/bin/bash
# head_score2 with staged LDS waits (FEDREC_HEAD_SCORE=7, since adopted as the default) vs the tiling
# without them (then the default, now FEDREC_HEAD_SCORE=2): text-head tests
# under the switch, then bench arms A/B/A/B.
source "$(dirname "$0")/../../gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
FEDREC_HEAD_SCORE=7 check t_hs 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_text_head_gpu.py tests/test_step_graph.py
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run b_def 200 $B
FEDREC_HEAD_SCORE=7 run b_hs 200 $B
run b_def2 200 $B
FEDREC_HEAD_SCORE=7 run b_hs2 200 $B
run b_def3 200 $B
FEDREC_HEAD_SCORE=7 run b_hs3 200 $B
for f in b_def b_hs b_def2 b_hs2 b_def3 b_hs3; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
O=$PWD/gpurun_out/prof_hs
rm -rf $O; mkdir -p $O
FEDREC_HEAD_SCORE=7 run prof_hs 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o hs -- python -u bench.py --steps 30 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 20 > gpurun_out/breakdown_hs.txt 2>&1
head -8 gpurun_out/breakdown_hs.txt
