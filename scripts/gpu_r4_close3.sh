#!/bin/bash
# closing check of the final tree: full GPU suite + smoke, bench (default / 50 steps)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_all 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
check smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 300 python -u bench.py
run bench50 300 python -u bench.py --steps 50
