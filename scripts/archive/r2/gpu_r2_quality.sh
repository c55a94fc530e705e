#!/bin/bash
# identity-scorer collapse diagnosis (verdict 8c) + the partial-tile GEMM tests
source "$(dirname "$0")/../../gpu_lib.sh"
check parttest 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_partial_gpu.py tests/test_kernels_gpu.py -m gpu
rm -f gpurun_out/quality_*.jsonl
run q_id_1e3 300 python benchmarks/quality_diag.py --lr 1e-3 --score-act identity --epochs 3 --out gpurun_out/quality_identity_lr1e-3.jsonl
run q_sig_1e3 300 python benchmarks/quality_diag.py --lr 1e-3 --score-act sigmoid --epochs 3 --out gpurun_out/quality_sigmoid_lr1e-3.jsonl
run q_id_5e5 300 python benchmarks/quality_diag.py --lr 5e-5 --score-act identity --epochs 3 --out gpurun_out/quality_identity_lr5e-5.jsonl
