"""Per-tile fixed cost of the ping-pong GEMM: the same M x N at K = 768 / 1536 / 3072, time =
a + b K per launch -> a / tiles is what a tile pays besides its k-steps (epilogue, tile switch).

    python benchmarks/gemm_k_sweep.py [out.jsonl]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fedrec_with_pytorchdistributed_amd.ops import native

lib = native.lib()
dev = torch.device("cuda")
out = open(sys.argv[1], "w") if len(sys.argv) > 1 else None


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


M = 409600
for N, act in ((2304, 0), (768, 0), (3072, 1)):
    res = {}
    for K in (768, 1536, 3072):
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        b = torch.rand(N, device=dev)
        for v in (-1, 9, 13):
            lib.gemm_set_variant(v)
            ms = timed(lambda: lib.linear(x, w, b, act, None))
            res[(K, v)] = ms
            rec = {"M": M, "N": N, "K": K, "act": act, "variant": v, "ms": round(ms, 4),
                   "TF": round(2.0 * M * N * K / ms / 1e9, 1)}
            print(json.dumps(rec), flush=True)
            if out:
                out.write(json.dumps(rec) + "\n")
        del x, w
    lib.gemm_set_variant(-1)
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    for v in (-1, 9, 13):
        t1, t2, t4 = res[(768, v)], res[(1536, v)], res[(3072, v)]
        slope = (t4 - t1) / (3072 - 768)
        a = t1 - slope * 768
        rec = {"N": N, "act": act, "variant": v, "fixed_ms": round(a, 4), "ms_per_k": round(slope * 1000, 5),
               "fixed_us_per_tile_per_cu": round(a * 1000 / (tiles / 256), 3),
               "fixed_share_at_K768": round(a / t1, 3)}
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
