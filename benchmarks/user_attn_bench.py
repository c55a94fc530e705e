"""User-encoder attention (20 heads x d_k 20, fp32) at the config-2 shape (B = 64 impressions,
H = 50 clicked news): forward and backward of the four-wave matrix-core kernels (median of
--rounds timings).

    python benchmarks/user_attn_bench.py [--out gpurun_out/user_attn_bench.json]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.ops import native


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--H", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lib = native.lib()
    NH, DK = 20, 20
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = torch.randn(a.B, a.H, 3 * NH * DK, generator=g).cuda()
    d = torch.randn(a.B, a.H, NH * DK, generator=g).cuda()
    c, st = ops.user_attention_fwd(qkv, NH, DK)
    res = {}
    times = {"fwd": [], "bwd": []}
    for _ in range(a.rounds):
        times["fwd"].append(timeit(lambda: ops.user_attention_fwd(qkv, NH, DK)))
        times["bwd"].append(timeit(lambda: ops.user_attention_bwd(qkv, st, d, NH, DK)))
    for k, v in times.items():
        res[k] = {"us": round(1000 * statistics.median(v), 2), "all_us": [round(1000 * x, 2) for x in v]}
        print(k, res[k], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
