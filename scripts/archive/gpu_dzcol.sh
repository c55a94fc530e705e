#!/bin/bash
# config 5: FFN1 bias gradient from the dF GEMM epilogue (column partials): numerics + A/B/A
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
run dztests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "linear_gelu_bwd or gelu_bwd or unfrozen"
run c5_d1 400 env FEDREC_DZ_MODE=stream python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_d0 400 env FEDREC_DZ_MODE=gemm python bench.py --config 5 --steps 10 --warmup 3 --no-valid
run c5_d1b 400 env FEDREC_DZ_MODE=stream python bench.py --config 5 --steps 10 --warmup 3 --no-valid
grep -h '^{' gpurun_out/c5_d1.log gpurun_out/c5_d0.log gpurun_out/c5_d1b.log > gpurun_out/dzcol_ab.jsonl || true
