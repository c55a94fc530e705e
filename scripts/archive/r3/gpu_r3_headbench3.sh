set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
run() { echo "== $*"; timeout -k 10 120 "$@" 2>&1 | grep -E "head_wgrad|head_score|head_pool|r2_|==" ; }
FEDREC_HEAD_WG=2 run python -u benchmarks/head_bench.py --iters 30 --N 1700
FEDREC_HEAD_WG=2 run python -u benchmarks/head_bench.py --iters 30 --N 20000
