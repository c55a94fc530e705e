set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_ipc_allreduce_gpu.py -x -v --timeout 200 --timeout-method thread 2>&1 | tail -15
