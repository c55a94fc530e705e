set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
mkdir -p gpurun_out
export FEDREC_ORACLE_ERRS=gpurun_out/r3_step_oracle_errors.json
timeout -k 10 900 python -u -m pytest tests/test_no_library_kernels_gpu.py tests/test_user_step_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_small_gemm_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/mask_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/mask_tests.log | tail -40; tail -60 gpurun_out/mask_tests.log; exit 1; }
grep -c PASSED gpurun_out/mask_tests.log; tail -3 gpurun_out/mask_tests.log
