#!/bin/bash
# closing sanity on the committed tree (the in-tree .so as the driver will load it): full GPU suite, smoke, bench
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_close 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
check smoke_close 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run r5close_c2 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
grep -o '"value": [0-9.]*\|"steady_ms_per_step": [0-9.]*' gpurun_out/r5close_c2.log
