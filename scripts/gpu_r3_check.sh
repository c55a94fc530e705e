set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_text_head_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_th_tests.log 2>&1 || { echo TESTFAIL; tail -50 gpurun_out/r3_th_tests.log; exit 1; }
tail -3 gpurun_out/r3_th_tests.log
timeout -k 10 300 python -u -m pytest tests/test_step_graph.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_eng_tests.log 2>&1 || { echo ENGFAIL; tail -50 gpurun_out/r3_eng_tests.log; exit 1; }
tail -3 gpurun_out/r3_eng_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench1.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/r3_bench1.log; exit 1; }
tail -3 gpurun_out/r3_bench1.log
