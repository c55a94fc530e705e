#!/bin/bash
# pruned tree (superseded kernels / switches removed, early user-slice reduce): full GPU suite + smoke + bench,
# then the federated quality runs with the server-step options and the final global-model score
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_r6f 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
check smoke_r6f 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run r6f_c2 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
run q_r6f 700 python -u scripts/quality_fed.py --out gpurun_out/r6_quality_fed2 --world 8 --only w8
tail -3 gpurun_out/t_r6f.log
grep -o '"value": [0-9.]*\|"steady_ms_per_step": [0-9.]*' gpurun_out/r6f_c2.log
cut -c1-300 gpurun_out/r6_quality_fed2/summary.jsonl
