"""Probe: time of one small_gemm launch vs K (k-steps) and M (blocks per CU) per tile variant,
bf16 operands -- separates per-k-step latency from per-launch overhead (diagnostic).  Tile 5 is
the 64 x 64 register-queue kernel, tile 1 the 64 x 64 LDS-DMA ring these launches take by
default; the last rows are the config-2 step's bf16 x bf16 forward shapes."""
import json
import sys

import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.ops import Gemm


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


dev = torch.device("cuda", 0)
out = []
shapes = [(M, N, K) for M, N in ((3200, 1200), (1600, 1200), (6400, 1200), (3200, 2400))
          for K in (64, 128, 256, 512, 1024)]
shapes += [(3200, 1200, 400), (3200, 200, 400), (1565, 400, 768), (64, 400, 400)]
for M, N, K in shapes:
    if True:
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        B = torch.randn(N, K, device=dev).to(torch.bfloat16)
        C = torch.zeros(M, N, device=dev)
        for tile in (5, 1, 4):
            g = Gemm(A, B, C, M, N, K, K, K, N)
            us = timeit(lambda: ops.small_gemm(g, tile=tile))
            rec = {"M": M, "N": N, "K": K, "tile": tile, "us": round(us, 2),
                   "TF": round(2.0 * M * N * K / us / 1e6, 1)}
            out.append(rec)
            print(json.dumps(rec), flush=True)
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
