#!/bin/bash
# head_score3 (X-only LDS ring, W1 fragments from L2): correctness, kernel A/B, step A/B;
# in-graph Adam; host timeline.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
FEDREC_HEAD_SCORE=8 check t_head8 300 $T tests/test_text_head_gpu.py
check t_graph 400 $T tests/test_step_graph.py tests/test_kernels_gpu.py -k "graph or user_attention or segment or dedup or score_ce"
for v in 7 8 7 8; do
  FEDREC_HEAD_SCORE=$v run hb_$v 120 python -u benchmarks/head_bench.py --iters 50
  grep head_score gpurun_out/hb_$v.log | sed "s/^/v=$v /" >> gpurun_out/hb_ab.txt
done
for v in 8 7 8 7; do
  FEDREC_HEAD_SCORE=$v run bn_$v 200 python -u bench.py --steps 50 --round off --no-valid
  echo "v=$v $(grep -o '"steady_ms_per_step": [0-9.]*' gpurun_out/bn_$v.log)" >> gpurun_out/bn_ab.txt
done
cat gpurun_out/hb_ab.txt gpurun_out/bn_ab.txt
run timeline 240 python -u benchmarks/host_timeline.py --steps 30 --json gpurun_out/host_timeline.json
tail -3 gpurun_out/timeline.log
check t_sg 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_small_gemm_gpu.py tests/test_user_step_gpu.py tests/test_engine_gpu.py
