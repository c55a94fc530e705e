#!/bin/bash
# config-5 iteration: kernel + engine GPU tests, config-5 bench, config-5 kernel profile
source "$(dirname "$0")/../../gpu_lib.sh"
check c5tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_wgrad_gpu.py -m gpu
run c5_ours 400 python bench.py --config 5 --steps 20 --warmup 5 --round off --no-valid
O=$PWD/gpurun_out/prof_c5
rm -rf $O; mkdir -p $O
run prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c5 -- python bench.py --config 5 --steps 6 --warmup 3 --round off --no-valid
