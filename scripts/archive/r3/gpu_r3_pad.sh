#!/bin/bash
# Padded-title skip (device nreal) in the text-head kernels: tests + config-2 bench A/B/A.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
check tests_pad 400 $T tests/test_text_head_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py tests/test_user_step_gpu.py tests/test_no_library_kernels_gpu.py tests/test_news_cache.py
check tests_dedup 200 $T tests/test_kernels_gpu.py -k dedup
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run bench_pad 200 $B
FEDREC_SKIP_PADDED=0 run bench_nopad 200 $B
run bench_pad2 200 $B
FEDREC_SKIP_PADDED=0 run bench_nopad2 200 $B
for f in bench_pad bench_nopad bench_pad2 bench_nopad2; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"], d["unique_titles_per_step"])')"; done
FEDREC_HEAD_SCORE=6 check oracle_s6 200 $T tests/test_text_head_gpu.py
FEDREC_HEAD_SCORE=6 run bench_s6 200 $B
run bench_pad3 200 $B
FEDREC_HEAD_SCORE=6 run bench_s6b 200 $B
for f in bench_s6 bench_pad3 bench_s6b; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"], d["unique_titles_per_step"])')"; done
