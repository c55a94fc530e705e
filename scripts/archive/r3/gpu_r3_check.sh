set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_text_head_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_tests.log 2>&1 || { echo TESTFAIL; tail -50 gpurun_out/r3_tests.log; exit 1; }
tail -2 gpurun_out/r3_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench1.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/r3_bench1.log; exit 1; }
tail -1 gpurun_out/r3_bench1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','steady_ms_per_step','round_s','round_impressions_per_s','valid_auc')})"
