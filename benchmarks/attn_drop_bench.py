"""Train-mode (dropout) title attention, forward and backward: the persistent prefetching
kernels (default) against the one-shot kernels, interleaved in one process at the config-5
shape (1,565 titles x 50 tokens, 12 heads).  Also checks that both forms give the same
outputs (same Philox mask, same math).

    python benchmarks/attn_drop_bench.py [--titles 1565] [--out gpurun_out/attn_drop.json]
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
    ap.add_argument("--titles", type=int, default=1565)
    ap.add_argument("--T", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lib = native.lib()
    dev = torch.device("cuda")
    n, T, D, H = a.titles, a.T, 768, 12
    M = n * T
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = (torch.randn(M, 3 * D, generator=g) * 0.5).to(dev, torch.bfloat16)
    dout = torch.randn(M, D, generator=g).to(dev, torch.bfloat16)
    lens = torch.randint(8, T + 1, (n,), generator=g)
    mask = (torch.arange(T)[None, :] < lens[:, None]).to(torch.int32).to(dev)
    p, seed, off = 0.1, 1234, 77

    def fwd(w):
        lib.title_attn_set_waves(w)
        return lib.title_attention_drop(qkv, mask, H, p, seed, off)

    def bwd(v, split=1):
        lib.title_attn_bwd_set_variant(10 + split)  # the dropout backward's prefetch form
        lib.title_attn_bwd_set_variant(v)
        return lib.title_attention_bwd_drop(qkv, dout, mask, H, p, seed, off)

    # same outputs from every form
    o_p, o_1 = fwd(-2).float(), fwd(2).float()
    g_p, g_1 = bwd(1).float(), bwd(0).float()
    g_n = bwd(1, 0).float()
    res = {"fwd_max_abs_diff": float((o_p - o_1).abs().max()),
           "bwd_max_abs_diff": float((g_p - g_1).abs().max()),
           "bwd_rel_l2": float((g_p - g_1).norm() / g_1.norm()),
           "bwd_split_vs_nosplit_max_abs_diff": float((g_p - g_n).abs().max())}
    print(res, flush=True)
    times = {"fwd_persistent": [], "fwd_oneshot": [], "bwd_persistent": [], "bwd_persistent_nosplit": [],
             "bwd_oneshot": []}
    for _ in range(a.rounds):
        times["fwd_persistent"].append(timeit(lambda: fwd(-2)))
        times["fwd_oneshot"].append(timeit(lambda: fwd(2)))
        times["bwd_persistent"].append(timeit(lambda: bwd(1)))
        times["bwd_persistent_nosplit"].append(timeit(lambda: bwd(1, 0)))
        times["bwd_oneshot"].append(timeit(lambda: bwd(0)))
    lib.title_attn_set_waves(-2)
    lib.title_attn_bwd_set_variant(11)
    lib.title_attn_bwd_set_variant(1)
    fbytes = M * 4 * D * 2  # read qkv, write out
    bbytes = M * 8 * D * 2  # read qkv + dout, write dqkv
    for k, v in times.items():
        ms = statistics.median(v)
        nb = fbytes if k.startswith("fwd") else bbytes
        res[k] = {"ms": round(ms, 4), "all_ms": [round(x, 4) for x in v], "GB/s": round(nb / ms / 1e6, 1)}
        print(k, res[k], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
