set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_small_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sg_tests.log 2>&1 || { tail -30 gpurun_out/sg_tests.log; exit 1; }
tail -3 gpurun_out/sg_tests.log

timeout -k 10 300 python -u benchmarks/small_gemm_bench.py --out gpurun_out/r3_small_gemm_bench.json > gpurun_out/sg_bench.log 2>&1 || { tail -30 gpurun_out/sg_bench.log; exit 1; }
cat gpurun_out/sg_bench.log
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 500 --timeout-method thread -k "two_clients" > gpurun_out/ipc2.log 2>&1 || { tail -40 gpurun_out/ipc2.log; exit 1; }
tail -8 gpurun_out/ipc2.log
