#!/bin/bash
# round-5 closing call: full GPU suite + smoke + bench configs 2 (driver default, 50 steps), 3, 4, 5
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_final 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
check smoke_final 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run r5final_c2 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
run r5final_c2_50 200 python -u bench.py --steps 50 --warmup 10
run r5final_c3 200 python -u bench.py --config 3
run r5final_c4 200 python -u bench.py --config 4
run r5final_c5 400 python -u bench.py --config 5
for f in gpurun_out/r5final_*.log; do echo $f $(grep -o '"steady_ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f); done
