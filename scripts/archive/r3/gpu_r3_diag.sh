#!/bin/bash
# Text-head diagnostics (gather vs contiguous, wgrad transform / split count) + score-tile bench A/B.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run diag_default 120 python -u benchmarks/head_diag.py
FEDREC_HEAD_WG=1 run diag_wg_notransform 120 python -u benchmarks/head_diag.py
FEDREC_HEAD_SPLITS=16 run diag_splits16 120 python -u benchmarks/head_diag.py
FEDREC_HEAD_SPLITS=60 run diag_splits60 120 python -u benchmarks/head_diag.py
FEDREC_HEAD_WG=6 run diag_w64 120 python -u benchmarks/head_diag.py
run bench_a 200 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
FEDREC_HEAD_SCORE=2 run bench_s2 200 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
run bench_a2 200 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
grep -h '^{' gpurun_out/diag_*.log > gpurun_out/diag_all.txt
for f in bench_a bench_s2 bench_a2; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
