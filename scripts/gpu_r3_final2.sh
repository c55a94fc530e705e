#!/bin/bash
# The new default-kernel test first, then the full verification (scripts/gpu_r3_final.sh).
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check t_defaults 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_no_library_kernels_gpu.py -k default_text_head
bash scripts/gpu_r3_final.sh
