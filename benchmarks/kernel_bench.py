"""Per-kernel microbenchmarks at the shapes of one training step (mind-small, B = 64 ->
~1577 unique titles x 50 tokens).  Reports median time, achieved HBM bandwidth (bytes the
kernel must move at minimum) and, for the MFMA kernels, TFLOP/s.

    python benchmarks/kernel_bench.py [--titles 1577] [--out gpurun_out/kernel_bench.json]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from fedrec_with_pytorchdistributed_amd.ops import native


def timeit(fn, iters=20, warm=3):
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
    ap.add_argument("--titles", type=int, default=1577)
    ap.add_argument("--T", type=int, default=50)
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lib = native.lib()
    dev = torch.device("cuda")
    n, T, D, H = a.titles, a.T, 768, 12
    M = n * T
    g = torch.Generator(device="cpu").manual_seed(0)
    res = {}

    def rec(name, ms, nbytes, flops=0.0):
        row = {"ms": round(ms, 4), "GB/s": round(nbytes / ms / 1e6, 1)}
        if flops:
            row["TFLOP/s"] = round(flops / ms / 1e9, 1)
        res[name] = row
        print(name, row, flush=True)

    want = lambda k: not a.only or k in a.only.split(",")
    qkv = (torch.randn(M, 3 * D, generator=g) * 0.5).to(dev, torch.bfloat16)
    lens = torch.randint(8, T + 1, (n,), generator=g)
    mask = (torch.arange(T)[None, :] < lens[:, None]).to(torch.int32).to(dev)
    if want("title_attention"):
        for w in (-2, -1, 0, 1, 2, 4):
            lib.title_attn_set_waves(w)
            ms = timeit(lambda: lib.title_attention(qkv, mask, H))
            rec(f"title_attention[{w}w]", ms, qkv.numel() * 2 + M * D * 2, 4.0 * n * H * T * T * 64)
        lib.title_attn_set_waves(-2)
    if want("packed"):
        # MIND-like title lengths ([CLS] + ~14 words + [SEP], synthetic generator's distribution)
        plens = (torch.randn(n, generator=g) * 5 + 16).round().clamp(5, 38).long()
        pmask = (torch.arange(T)[None, :] < plens[:, None]).to(torch.int32).to(dev)
        ms = timeit(lambda: lib.title_plan(pmask))
        rec("title_plan", ms, pmask.numel() * 4 * 3)
        rowmap, src, kv_start, kv_len, qstart, n_kv = lib.title_plan(pmask)
        R = int(n_kv.item())
        ms = timeit(lambda: lib.title_attention_packed(qkv, rowmap, kv_start, kv_len, qstart, H))
        rec("title_attention_packed", ms, M * D * 2 + R * 2 * D * 2 + M * D * 2,
            4.0 * H * 64 * float((plens * T).sum()))
        for w in (-2,):
            lib.title_attn_set_waves(w)
            ms = timeit(lambda: lib.title_attention(qkv, pmask, H))
            rec("title_attention_unpacked_same_lengths", ms, qkv.numel() * 2 + M * D * 2, 4.0 * n * H * T * T * 64)
        xin = (torch.randn(M, D, generator=g) * 0.5).to(dev, torch.bfloat16)
        wq = (torch.randn(3 * D, D, generator=g) * 0.03).to(dev, torch.bfloat16)
        bq = torch.randn(3 * D, device=dev)
        ms = timeit(lambda: lib.linear_split(xin, wq, bq, n_kv, D))
        rec("qkv_linear_split", ms, 0, 2.0 * D * (R * 3 * D + (M - R) * D))
        ms = timeit(lambda: lib.linear(xin, wq, bq, 0, None))
        rec("qkv_linear_full", ms, 0, 2.0 * M * D * 3 * D)
    if want("title_attention_bwd"):
        dout = (torch.randn(M, D, generator=g) * 0.1).to(dev, torch.bfloat16)
        ms = timeit(lambda: lib.title_attention_bwd(qkv, dout, mask, H))
        rec("title_attention_bwd", ms, qkv.numel() * 4 + M * D * 2, 8.0 * n * H * T * T * 64)
    x = (torch.randn(M, D, generator=g)).to(dev, torch.bfloat16)
    w, b = torch.randn(D, device=dev), torch.randn(D, device=dev)
    if want("layer_norm"):
        for wide in (0, 1):
            lib.ln_set_wide(wide)
            ms = timeit(lambda: lib.layer_norm(x, w, b, 1e-12))
            rec(f"layer_norm[wide={wide}]", ms, 2 * M * D * 2)
        lib.ln_set_wide(1)
        r = torch.randn(M, D, generator=g).to(dev, torch.bfloat16)
        for wide in (0, 1, 2, 3):  # 1/2/3: half-wave rows, 2/1/4 rows per half-wave
            lib.ln_set_wide(wide)
            ms = timeit(lambda: lib.layer_norm(x, w, b, 1e-12, r))
            rec(f"layer_norm+residual[wide={wide}]", ms, 3 * M * D * 2)
        lib.ln_set_wide(1)
    if want("embed_ln"):
        word = (torch.randn(30522, D, generator=g) * 0.02).to(dev, torch.bfloat16)
        pos = (torch.randn(512, D, generator=g) * 0.02).to(dev, torch.bfloat16)
        tok = torch.randint(0, 30522, (n, T), generator=g, dtype=torch.int32).to(dev)
        for wide in (0, 1):
            lib.ln_set_wide(wide)
            ms = timeit(lambda: lib.embed_ln(tok, word, pos, w, b, 1e-12))
            rec(f"embed_ln[wide={wide}]", ms, 2 * M * D * 2)
        lib.ln_set_wide(1)
    if want("additive_pool"):
        from fedrec_with_pytorchdistributed_amd import ops
        xh = x.view(n, T, D)
        e = torch.tanh(torch.randn(n, T, 384, generator=g)).to(dev, torch.bfloat16)
        w2 = torch.randn(384, device=dev) * 0.1
        b2 = torch.randn(1, device=dev)
        ms = timeit(lambda: ops.additive_pool_fwd(xh, e, w2, b2))
        rec("additive_pool_fwd", ms, x.numel() * 2 + e.numel() * 2)
        _, alpha = ops.additive_pool_fwd(xh, e, w2, b2)
        gg = torch.randn(n, D, device=dev)
        ms = timeit(lambda: ops.additive_pool_bwd(xh, e, alpha, w2, gg, False))
        rec("additive_pool_bwd", ms, x.numel() * 2 + e.numel() * 4)
    if want("wgrad"):
        from fedrec_with_pytorchdistributed_amd.ops.functional import wgrad
        dy = torch.randn(M, 384, generator=g).to(dev, torch.bfloat16)
        ms = timeit(lambda: wgrad(dy, x))
        rec("wgrad_splitk", ms, dy.numel() * 2 + x.numel() * 2, 2.0 * M * 384 * D)
        ms = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        rec("wgrad_mm", ms, dy.numel() * 2 + x.numel() * 2, 2.0 * M * 384 * D)
    if want("train"):  # unfrozen-backbone reductions (config 5)
        for N in (768, 2304, 3072):
            dyb = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
            ms = timeit(lambda: lib.colsum(dyb))
            rec(f"colsum[N={N}]", ms, dyb.numel() * 2)
            ms = timeit(lambda: dyb.sum(0, dtype=torch.float32))
            rec(f"torch_sum[N={N}]", ms, dyb.numel() * 2)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
