#!/bin/bash
# Segment sum with 8-occurrence chunks (default) vs 16 (FEDREC_SEGSUM_SCH=16): tests + bench A/B/A/B.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
check seg_tests 300 $T tests/test_kernels_gpu.py -k "segment or dedup or ldp"
FEDREC_SEGSUM_SCH=16 check seg_tests16 300 $T tests/test_kernels_gpu.py -k "segment"
check seg_tests2 300 $T tests/test_user_step_gpu.py tests/test_engine_gpu.py tests/test_step_graph.py
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run s_8a 200 $B
FEDREC_SEGSUM_SCH=16 run s_16a 200 $B
run s_8b 200 $B
FEDREC_SEGSUM_SCH=16 run s_16b 200 $B
for f in s_8a s_16a s_8b s_16b; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
# user attention: 64-row stages / PLDB 66 (default) vs the first LDS sizing (FEDREC_UA_VARIANT=4)
check ua_tests 300 $T tests/test_kernels_gpu.py -k "user_attention"
run ua_bench 200 python -u benchmarks/user_attn_bench.py --out gpurun_out/r3_user_attn_lds_bench.json
FEDREC_UA_VARIANT=4 run u_4a 200 $B
run u_3a 200 $B
FEDREC_UA_VARIANT=4 run u_4b 200 $B
run u_3b 200 $B
for f in u_4a u_3a u_4b u_3b; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
python -c "import json; d=json.load(open('gpurun_out/r3_user_attn_lds_bench.json')); print({k: v['us'] if isinstance(v, dict) else v for k, v in d.items()})"
