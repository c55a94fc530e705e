set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c2 -o c2 -- python -u bench.py --steps 30 --warmup 5 --round off --no-valid > gpurun_out/r3_prof_bench.log 2>&1 || { echo PROFFAIL; tail -30 gpurun_out/r3_prof_bench.log; exit 1; }
tail -2 gpurun_out/r3_prof_bench.log
f=$(find gpurun_out/prof_c2 -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 20 --json gpurun_out/r3_c2_breakdown.json | head -40
