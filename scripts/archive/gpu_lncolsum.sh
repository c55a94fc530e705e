#!/bin/bash
# config 5: LN backward also emits the bias gradient of the block feeding it (A/B/A)
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run lctests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "layer_norm_bwd or unfrozen"
run c5_f1 400 env FEDREC_LN_COLSUM=1 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_f0 400 env FEDREC_LN_COLSUM=0 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_f1b 400 env FEDREC_LN_COLSUM=1 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
grep -h '^{' gpurun_out/c5_f1.log gpurun_out/c5_f0.log gpurun_out/c5_f1b.log > gpurun_out/lncolsum_ab.jsonl || true
