#!/bin/bash
# checkpoint: full GPU suite + smoke + configs 2 / 4 (driver default) + config 2 at 50 steps
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_all_ae 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
check smoke_ae 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run r5ae_bench 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
run r5ae_bench_c4 200 python -u bench.py --config 4
run r5ae_bench_50 200 python -u bench.py --steps 50 --warmup 10
