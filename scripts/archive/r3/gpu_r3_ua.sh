set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "user_attention" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
timeout -k 10 120 python -u benchmarks/user_attn_bench.py --out gpurun_out/r3_user_attn_mfma_bench.json 2>&1 | tail -8 || exit 1
