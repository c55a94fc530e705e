#!/bin/bash
# User attention with smaller LDS stages (fwd 5 blocks/CU, bwd 3): oracle tests, kernel bench,
# config-2 bench arms (compare with r3_ab_casts_knobs.txt's k_def 0.5672 / 0.5674 ms).
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
check ua_tests 300 $T tests/test_kernels_gpu.py -k "user_attention or user_attn"
check ua_tests2 300 $T tests/test_user_step_gpu.py tests/test_engine_gpu.py
run ua_bench 200 python -u benchmarks/user_attn_bench.py --out gpurun_out/r3_user_attn_lds_bench.json
B="python -u bench.py --steps 50 --warmup 10 --round off --no-valid"
run u_a 200 $B
run u_b 200 $B
run u_c 200 $B
for f in u_a u_b u_c; do echo "$f $(tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["steady_ms_per_step"])')"; done
python -c "import json; d=json.load(open('gpurun_out/r3_user_attn_lds_bench.json')); print({k: v['us'] if isinstance(v, dict) else v for k, v in d.items()})"
