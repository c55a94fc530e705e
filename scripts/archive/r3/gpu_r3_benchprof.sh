set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench1.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/r3_bench1.log; exit 1; }
tail -1 gpurun_out/r3_bench1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','steady_ms_per_step','round_s','round_impressions_per_s','valid_auc')})"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c2 -o c2 -- python -u bench.py --steps 30 --warmup 5 --round off --no-valid > gpurun_out/r3_prof_bench.log 2>&1 || { echo PROFFAIL; tail -30 gpurun_out/r3_prof_bench.log; exit 1; }
f=$(find gpurun_out/prof_c2 -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 20 --json gpurun_out/r3_c2_breakdown.json | head -45
