#!/bin/bash
# tree with head_score2's interleaved issue as the default and the tr_read2 early-clobber fix:
# full GPU suite + smoke + driver-default bench + a 50-step bench
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_r6n 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
check smoke_r6n 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run r6n_c2 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
run r6n_c2_50 200 python -u bench.py --gpus 1 --steps 50 --warmup 10 --no-probe
tail -3 gpurun_out/t_r6n.log
grep -o '"value": [0-9.]*\|"steady_ms_per_step": [0-9.]*' gpurun_out/r6n_c2.log gpurun_out/r6n_c2_50.log
