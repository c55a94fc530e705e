#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_graph_ar 600 python -u -m pytest tests/test_multirank_gpu.py -k "graph_allreduce or bench_two" -x -v --timeout 400 --timeout-method thread -p no:cacheprovider
run r5b_bench2 300 python -u -c "
import sys; sys.path.insert(0,'tests')
from launch_util import run_ranks
SHARE={'FEDREC_CPU_ONLY':'0','FEDREC_SHARE_GPU':'1','FEDREC_DATA_BACKEND':'gloo','FEDREC_QUIET':'1'}
outs=run_ranks([['bench.py','--gpus','2','--steps','20','--warmup','5']]*2, SHARE, timeout=280)
for rc,out in outs: print(rc); print(out[-3000:])
"
run r5b_bench 300 python -u bench.py
