"""Diagnostics for the fused text-head kernels (csrc/text_head.hip) at the config-2 shape:
the same kernels on (a) the hidden-state cache through the title index (the step's form) and
(b) a materialised contiguous copy of the gathered rows (ids = None), so the cost of the
per-row gather shows directly; the wgrad also without its e -> g transform
(FEDREC_HEAD_WG=1 must be set in the environment for that arm: the switch is read once).

    python benchmarks/head_diag.py [--U 1600] [--N 65000]
"""
import argparse
import json
import math
import os

import torch

from fedrec_with_pytorchdistributed_amd.ops import native


def timeit(fn, iters):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--U", type=int, default=1600)
    ap.add_argument("--N", type=int, default=65000)
    ap.add_argument("--T", type=int, default=50)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    D, Q, T, U = 768, 384, a.T, a.U
    g = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(a.N * T, D, device=dev, generator=g).to(torch.bfloat16)
    ids = torch.randperm(a.N, device=dev, generator=g)[:U].to(torch.int32)
    w1 = (torch.randn(Q, D, device=dev, generator=g) / math.sqrt(D)).to(torch.bfloat16)
    b1 = torch.randn(Q, device=dev, generator=g) * 0.1
    w2 = torch.randn(Q, device=dev, generator=g) / math.sqrt(Q)
    b2 = torch.zeros(1, device=dev)
    lib = native.lib()
    M = U * T
    hid = table.view(a.N, T, D).index_select(0, ids.long()).reshape(M, D).contiguous()
    tag = {k: v for k, v in os.environ.items() if k.startswith("FEDREC_HEAD")}
    for name, tab, ix in (("gather", table, ids), ("contig", hid, None)):
        e, sc = lib.head_score(tab, ix, T, w1, b1, w2, b2, True)
        pooled, alpha, _ = lib.head_pool(tab, ix, T, sc, None)
        gout = torch.randn(U, D, device=dev, generator=g)
        da, db2p = lib.head_pool_bwd(tab, ix, T, alpha, gout)
        res = {"src": name, "env": tag}
        res["score_us"] = round(timeit(lambda: lib.head_score(tab, ix, T, w1, b1, w2, b2, True), a.iters), 1)
        res["score_noe_us"] = round(timeit(lambda: lib.head_score(tab, ix, T, w1, b1, w2, b2, False), a.iters), 1)
        res["pool_us"] = round(timeit(lambda: lib.head_pool(tab, ix, T, sc, None), a.iters), 1)
        res["pool_bwd_us"] = round(timeit(lambda: lib.head_pool_bwd(tab, ix, T, alpha, gout), a.iters), 1)
        res["wgrad_us"] = round(timeit(lambda: lib.head_wgrad(tab, ix, T, e, da, w2, db2p), a.iters), 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
