#!/bin/bash
# config 5: QKV bias gradient from the dQ slice + identities (dV sum = dbo Wo, dK sum = 0): A/B/A
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run qbtests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "colsum or unfrozen"
run c5_q1 400 env FEDREC_QKV_BIAS_SHORTCUT=1 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_q0 400 env FEDREC_QKV_BIAS_SHORTCUT=0 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_q1b 400 env FEDREC_QKV_BIAS_SHORTCUT=1 python bench.py --config 5 --steps 10 --warmup 3 --no-valid
grep -h '^{' gpurun_out/c5_q1.log gpurun_out/c5_q0.log gpurun_out/c5_q1b.log > gpurun_out/qkvbias_ab.jsonl || true
