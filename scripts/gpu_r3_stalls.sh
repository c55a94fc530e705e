#!/bin/bash
# Wave-state counters of the config-2 step (two --pmc passes of 8 SQ counters each, each pass
# its own run of the same short bench) -> benchmarks/pmc_stalls.py; then the staged-wait
# head_wgrad (FEDREC_HEAD_WG=16 = then the staged waits; since their adoption the single-wait form) bench arms again, and the step counter advanced in the cast
# launch (default) vs a torch add_ (FEDREC_STEP_BUMP=0).
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/pmc_stalls
rm -rf "$O"; mkdir -p "$O"
check t_mcast 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k multi_cast
check t_bump 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_step_graph.py tests/test_engine_gpu.py
B="python -u bench.py --steps 20 --warmup 5 --round off --no-valid"
run pmc_s1 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC -- $B
run pmc_s2 200 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O" -o s2 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES -- $B
python benchmarks/pmc_stalls.py "$O" > gpurun_out/r3_pmc_stalls.json
head -c 2500 gpurun_out/r3_pmc_stalls.json
B2="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run b_def 200 $B2
FEDREC_HEAD_WG=16 run b_sw 200 $B2
run b_def2 200 $B2
FEDREC_HEAD_WG=16 run b_sw2 200 $B2
FEDREC_STEP_BUMP=0 run b_nobump 200 $B2
FEDREC_STEP_BUMP=0 run b_nobump2 200 $B2
for f in b_def b_sw b_def2 b_sw2 b_nobump b_nobump2; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
