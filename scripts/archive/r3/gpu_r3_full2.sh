set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_small_gemm_gpu.py tests/test_no_library_kernels_gpu.py tests/test_user_step_gpu.py tests/test_engine_gpu.py tests/test_step_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { grep -E "^E |FAIL" gpurun_out/full_tests.log | head -30; tail -30 gpurun_out/full_tests.log; exit 1; }
tail -1 gpurun_out/full_tests.log
bash scripts/gpu_r3_benchprof.sh
