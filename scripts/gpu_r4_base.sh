#!/bin/bash
# Round-4 opening measurement: smoke, the driver-default bench, the GEMM bench against
# hipBLASLt at the DistilBERT shapes, and a kernel trace of the config-2 bench (cache build
# + step).
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
check smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python -u bench.py
run gemm 400 python -u benchmarks/gemm_bench.py --rounds 5 --out gpurun_out/r4_gemm_bench_base.json
O=$PWD/gpurun_out/prof_c2
rm -rf $O; mkdir -p $O
run prof_c2 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_base.json > gpurun_out/breakdown_c2.txt 2>&1
python benchmarks/phase_breakdown.py "$f" --until sample_kernel --json gpurun_out/r4_cache_build_base.json > gpurun_out/cache_build.txt 2>&1
head -30 gpurun_out/cache_build.txt
