#!/bin/bash
# which hipBLASLt kernels (tile / workgroup config in the name) win at 8192^3 and at the build's shapes
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/prof_r5y
rm -rf $O; mkdir -p $O
run prof_r5y_sq 300 rocprofv3 --kernel-trace --output-format csv -d $O -o sq -- python -u benchmarks/gemm_bench.py --shapes square --rounds 3
run prof_r5y_m 300 rocprofv3 --kernel-trace --output-format csv -d $O -o m -- python -u benchmarks/gemm_bench.py --M 409600 --rounds 3
python - "$O" <<'PY' > gpurun_out/r5y_gemm_kernels.txt
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        a = agg[n]; a[0] += 1; a[1] += d
    print("==", f)
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:14]:
        print(f"{t/c:10.1f} us x{c:4d}  {n[:230]}")
PY
cat gpurun_out/r5y_gemm_kernels.txt | head -40
grep -h "TF\|tflops\|{" gpurun_out/prof_r5y_sq.log | tail -5
