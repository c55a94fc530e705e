#!/bin/bash
# persistent LayerNorm (variant 4) vs the one-shot default: kernel A/B + whole-step A/B in one call
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run lntests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "layer_norm"
run ln_ab 300 python benchmarks/ln_ab.py
for i in 1 2; do
  run b_ln1_$i 300 env FEDREC_LN_WIDE=1 python bench.py --config 2 --steps 30 --warmup 5 --no-valid
  run b_ln4_$i 300 env FEDREC_LN_WIDE=4 python bench.py --config 2 --steps 30 --warmup 5 --no-valid
done
run packed4 300 env FEDREC_LN_WIDE=4 python -u -m pytest tests/test_packed_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread
grep -h '^{' gpurun_out/b_ln*.log > gpurun_out/ln_ab_bench.jsonl || true
