#!/bin/bash
# checkpoint: full GPU suite + smoke + config-2 / config-4 bench (driver default)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_all 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
check smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run r5x_bench 200 python -u bench.py
run r5x_bench_c4 200 python -u bench.py --config 4
