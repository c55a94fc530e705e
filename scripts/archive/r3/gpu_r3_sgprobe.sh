set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/sg_latency_probe.py gpurun_out/sg_probe.json > gpurun_out/sg_probe.log 2>&1 || { tail -30 gpurun_out/sg_probe.log; exit 1; }
cat gpurun_out/sg_probe.log
