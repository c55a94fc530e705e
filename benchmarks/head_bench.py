"""Per-kernel timing of the fused text head (csrc/text_head.hip) at the config-2 step shape:
a MIND-small-sized hidden-state cache [N, 50, 768] bf16 in HBM and U unique titles per step.

    python benchmarks/head_bench.py [--U 1600] [--N 65000] [--iters 50]

Prints one JSON line per kernel: us per call and achieved TF/s (GEMM kernels) or TB/s
(streaming kernels, algorithmic bytes)."""
import argparse
import json
import math

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
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--ids", default="perm", choices=["perm", "sorted", "pool64", "same"],
                    help="which cache titles a step reads: random (perm, the real case), random sorted, "
                         "64 distinct titles (L2 / Infinity-Cache resident) or one title: where the X "
                         "rows are served from, to tell fetch-bound from compute-bound kernels")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    D, Q, T, U = 768, 384, a.T, a.U
    g = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(a.N * T, D, device=dev, generator=g).to(torch.bfloat16)
    ids = torch.randperm(a.N, device=dev, generator=g)[:U].to(torch.int32)
    if a.ids == "sorted":
        ids = ids.sort().values
    elif a.ids == "pool64":
        ids = ids[:64].repeat((U + 63) // 64)[:U].contiguous()
    elif a.ids == "same":
        ids = ids[:1].repeat(U).contiguous()
    w1 = (torch.randn(Q, D, device=dev, generator=g) / math.sqrt(D)).to(torch.bfloat16)
    b1 = torch.randn(Q, device=dev, generator=g) * 0.1
    w2 = torch.randn(Q, device=dev, generator=g) / math.sqrt(Q)
    b2 = torch.zeros(1, device=dev)
    lib = native.lib()
    M = U * T
    e, sc = lib.head_score(table, ids, T, w1, b1, w2, b2, True)
    pooled, alpha, _ = lib.head_pool(table, ids, T, sc, None)
    gout = torch.randn(U, D, device=dev, generator=g)
    da, db2p = lib.head_pool_bwd(table, ids, T, alpha, gout)
    out = []
    t = timeit(lambda: lib.head_score(table, ids, T, w1, b1, w2, b2, True), a.iters)
    out.append({"kernel": "head_score", "us": round(t, 1), "TFs": round(2 * M * Q * D / t / 1e6, 1), "ids": a.ids})
    for rows in (192, 160):  # the row tile forced (the default picks by the rounds rule)
        for ilv in (0, 1):
            lib.head_score_set_rows(rows)
            lib.head_score_set_ilv(ilv)
            t = timeit(lambda: lib.head_score(table, ids, T, w1, b1, w2, b2, True), a.iters)
            out.append({"kernel": f"head_score_{rows}rows_ilv{ilv}", "us": round(t, 1),
                        "TFs": round(2 * M * Q * D / t / 1e6, 1)})
    lib.head_score_set_rows(0)
    lib.head_score_set_ilv(1)
    t = timeit(lambda: lib.head_pool(table, ids, T, sc, None), a.iters)
    out.append({"kernel": "head_pool", "us": round(t, 1), "TBs": round(M * D * 2 / t / 1e6, 2)})
    t = timeit(lambda: lib.head_pool_bwd(table, ids, T, alpha, gout), a.iters)
    out.append({"kernel": "head_pool_bwd", "us": round(t, 1), "TBs": round(M * D * 2 / t / 1e6, 2)})
    t = timeit(lambda: lib.head_wgrad(table, ids, T, e, da, w2, db2p), a.iters)
    out.append({"kernel": "head_wgrad(+reduce)", "us": round(t, 1), "TFs": round(2 * M * Q * D / t / 1e6, 1)})
    # the G path (round 5): g = da (1 - e^2) written once by the pool backward, then a plain TN
    # GEMM over g
    if lib.head_g_supported(D, Q, T):
        eg = e.clone()
        t = timeit(lambda: lib.head_pool_bwd_g(table, ids, T, alpha, gout, eg), a.iters)
        out.append({"kernel": "head_pool_bwd_g (fused)", "us": round(t, 1),
                    "TBs": round(M * (D + 2 * Q) * 2 / t / 1e6, 2)})
        eg.copy_(e)
        _, _, cs = lib.head_pool_bwd_g(table, ids, T, alpha, gout, eg)
        t = timeit(lambda: lib.head_wgrad_g(table, ids, T, eg, cs, w2, db2p), a.iters)
        out.append({"kernel": "head_wgrad_g(+reduce)", "us": round(t, 1), "TFs": round(2 * M * Q * D / t / 1e6, 1)})
    # the round-2 pieces for reference: gather + plain GEMM + wgrad of a materialised dpre
    hid = table.view(a.N, T, D).index_select(0, ids.long()).reshape(M, D)
    t = timeit(lambda: table.view(a.N, T, D).index_select(0, ids.long()), a.iters)
    out.append({"kernel": "r2_gather", "us": round(t, 1)})
    t = timeit(lambda: lib.linear(hid, w1, b1, 2, None), a.iters)
    out.append({"kernel": "r2_gemm_tanh", "us": round(t, 1), "TFs": round(2 * M * Q * D / t / 1e6, 1)})
    dpre = e.clone()
    t = timeit(lambda: lib.wgrad(dpre, hid), a.iters)
    out.append({"kernel": "r2_wgrad", "us": round(t, 1), "TFs": round(2 * M * Q * D / t / 1e6, 1)})
    for r in out:
        r.update({"U": U, "T": T, "M": M})
        print(json.dumps({**r, "ids": a.ids}), flush=True)


if __name__ == "__main__":
    main()
