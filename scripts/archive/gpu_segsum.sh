#!/bin/bash
# chunked deterministic segment sum: numerics, kernel time, whole-step A/B
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run sstests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "segment_sum or dedup or ldp or oracle or per_epoch"
for i in 1 2; do
  run s1_$i 300 env FEDREC_SEGSUM_VARIANT=1 python bench.py --config 2 --steps 40 --warmup 5 --no-valid
  run s0_$i 300 env FEDREC_SEGSUM_VARIANT=0 python bench.py --config 2 --steps 40 --warmup 5 --no-valid
done
grep -h '^{' gpurun_out/s1_*.log gpurun_out/s0_*.log > gpurun_out/segsum_ab.jsonl || true
O=$PWD/gpurun_out/prof_ss
mkdir -p $O
run profss 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o ss -- python bench.py --config 2 --steps 10 --warmup 3 --no-valid
