set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py tests/test_engine_gpu.py tests/test_step_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sg_tests.log 2>&1 || { tail -40 gpurun_out/sg_tests.log; exit 1; }
tail -3 gpurun_out/sg_tests.log
timeout -k 10 300 python -u benchmarks/small_gemm_bench.py --out gpurun_out/r3_small_gemm_bench.json > gpurun_out/sg_bench.log 2>&1 || { tail -30 gpurun_out/sg_bench.log; exit 1; }
grep -v '"tile": [234]' gpurun_out/sg_bench.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench1.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/r3_bench1.log; exit 1; }
tail -1 gpurun_out/r3_bench1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','steady_ms_per_step','round_s','round_impressions_per_s','valid_auc')})"
