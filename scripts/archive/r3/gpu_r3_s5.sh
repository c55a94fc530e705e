#!/bin/bash
# Round-3 head/user-side A/B: Q-sliced score (5), interleaved wgrad transform (default; 8 = old),
# side-stream weight gradients (default; FEDREC_SIDE_GRADS=0 = inline): tests, head diag, bench.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
check tests_def 400 $T tests/test_text_head_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py tests/test_user_step_gpu.py tests/test_no_library_kernels_gpu.py
FEDREC_HEAD_SCORE=5 check oracle_s5 200 $T tests/test_text_head_gpu.py
run diag_def 120 python -u benchmarks/head_diag.py
FEDREC_HEAD_SCORE=5 run diag_s5 120 python -u benchmarks/head_diag.py
FEDREC_HEAD_WG=8 run diag_wg8 120 python -u benchmarks/head_diag.py
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run bench_a 200 $B
FEDREC_SIDE_GRADS=0 run bench_noside 200 $B
FEDREC_HEAD_SCORE=5 run bench_s5 200 $B
FEDREC_HEAD_WG=8 run bench_wg8 200 $B
run bench_a2 200 $B
grep -h '^{' gpurun_out/diag_def.log gpurun_out/diag_s5.log gpurun_out/diag_wg8.log
for f in bench_a bench_noside bench_s5 bench_wg8 bench_a2; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
