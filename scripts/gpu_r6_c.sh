#!/bin/bash
# early user-slice reduce at N > 1: multi-rank GPU tests (shared-GPU rehearsal), the 2-client
# kernel trace (launch order), then the N = 1 step A/B is unaffected (no all-reduce at N = 1)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_multirank 900 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -k "graph_allreduce or ipc"
O=$PWD/gpurun_out/prof_r6c; rm -rf $O; mkdir -p $O
run prof_r6c 400 rocprofv3 --kernel-trace --output-format csv -d $O -o %pid%_tr -- python -u benchmarks/early_reduce_trace.py 2
ls $O
for f in $(find $O -name "*kernel_trace.csv"); do echo "== $f"; python benchmarks/early_reduce_order.py $f --json ${f%.csv}_early.json | tail -4; done
check t_engine 600 python -u -m pytest tests/test_engine_gpu.py tests/test_step_graph.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
run r6c_c2 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
