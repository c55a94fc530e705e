set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 500 --timeout-method thread -k "two_clients" 2>&1 | tail -15
