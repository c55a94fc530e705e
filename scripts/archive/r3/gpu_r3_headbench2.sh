set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
timeout -k 10 200 python -u -m pytest tests/test_text_head_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
run() { echo "== $*"; timeout -k 10 120 "$@" 2>&1 | grep -E "head_|==" ; }
run python -u benchmarks/head_bench.py --iters 30
FEDREC_HEAD_WG=2 run python -u benchmarks/head_bench.py --iters 30
FEDREC_HEAD_SPLITS=40 run python -u benchmarks/head_bench.py --iters 30
