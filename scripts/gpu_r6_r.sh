#!/bin/bash
# HIP runtime switches vs the graph-boundary cost (benchmarks/graph_boundary.py, 20 small kernels)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run gb_default 100 python -u benchmarks/graph_boundary.py --numel 65536 --kernels 10
run gb_pc0 100 env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python -u benchmarks/graph_boundary.py --numel 65536 --kernels 10
run gb_pc1 100 env DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 python -u benchmarks/graph_boundary.py --numel 65536 --kernels 10
run gb_hdp0 100 env DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0 python -u benchmarks/graph_boundary.py --numel 65536 --kernels 10
run gb_sys0 100 env ROC_SYSTEM_SCOPE_SIGNAL=0 python -u benchmarks/graph_boundary.py --numel 65536 --kernels 10
run gb_devka 100 env HIP_FORCE_DEV_KERNARG=1 python -u benchmarks/graph_boundary.py --numel 65536 --kernels 10
for f in gpurun_out/gb_*.log; do echo "$f"; grep '"mode"' "$f" | head -3; done
