#!/bin/bash
# pool backward + g rewrite in one launch (e loaded after the X rows): tests, then A/B/A/B at 50 steps
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_ad 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_text_head_gpu.py
run r5ad_new1 200 env FEDREC_HEAD_G_FUSED=1 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
run r5ad_old1 200 env FEDREC_HEAD_G_FUSED=0 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
run r5ad_new2 200 env FEDREC_HEAD_G_FUSED=1 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
run r5ad_old2 200 env FEDREC_HEAD_G_FUSED=0 python -u bench.py --steps 50 --warmup 10 --round off --no-valid
O=$PWD/gpurun_out/prof_ad; rm -rf $O; mkdir -p $O
run prof_ad 200 env FEDREC_HEAD_G_FUSED=1 rocprofv3 --kernel-trace --output-format csv -d $O -o ad -- python -u bench.py --steps 10 --warmup 5 --round off --no-valid
for f in gpurun_out/r5ad_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f); done
