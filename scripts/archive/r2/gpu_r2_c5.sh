#!/bin/bash
# config 5 on our backward GEMMs: GPU tests that train the unfrozen backbone, config-5 A/B
# (library dX/dW vs ours), a config-5 kernel profile
source "$(dirname "$0")/../../gpu_lib.sh"
check c5tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_wgrad_gpu.py tests/test_kernels_gpu.py tests/test_dropout.py -m gpu
rm -f gpurun_out/c5_ab.jsonl
run c5_ours 400 python bench.py --config 5 --steps 20 --warmup 5 --round off --no-valid
grep -h '^{' gpurun_out/c5_ours.log | sed 's/^{/{"arm": "ours", /' >> gpurun_out/c5_ab.jsonl || true
FEDREC_DGRAD=lib FEDREC_WGRAD=lib run c5_lib 400 python bench.py --config 5 --steps 20 --warmup 5 --round off --no-valid
grep -h '^{' gpurun_out/c5_lib.log | sed 's/^{/{"arm": "lib", /' >> gpurun_out/c5_ab.jsonl || true
O=$PWD/gpurun_out/prof_c5
rm -rf $O; mkdir -p $O
run prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c5 -- python bench.py --config 5 --steps 6 --warmup 3 --round off --no-valid
