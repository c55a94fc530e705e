#!/bin/bash
# Existing A/B knobs re-checked on the current step (config 2, 50-step arms): small-GEMM tile
# forced to 128x64 / 64x128 / 128x128, one-wave MFMA user attention, block-per-row segment sum.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
check k_tests 400 $T tests/test_step_graph.py tests/test_engine_gpu.py tests/test_user_step_gpu.py tests/test_no_library_kernels_gpu.py tests/test_text_head_gpu.py
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run k_def 200 $B
FEDREC_STEP_CASTS=0 run k_nocast 200 $B
FEDREC_SG_TILE=2 run k_sg2 200 $B
FEDREC_SG_TILE=3 run k_sg3 200 $B
FEDREC_SG_TILE=4 run k_sg4 200 $B
FEDREC_UA_VARIANT=2 run k_ua2 200 $B
FEDREC_SEGSUM_VARIANT=0 run k_seg0 200 $B
run k_def2 200 $B
FEDREC_STEP_CASTS=0 run k_nocast2 200 $B
for f in k_def k_nocast k_sg2 k_sg3 k_sg4 k_ua2 k_seg0 k_def2 k_nocast2; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
