"""GEMM microbenchmark at the DistilBERT shapes of one training step (M = unique titles x 50).

Interleaves every variant in ONE process (cdna_hip_programming.md §5.4 rule 24) on random
data (rule 25) and reports the median TFLOP/s per variant:
  ours-128   : 128x128x64 tile, 4 waves, glds double buffer
  ours-pp-v6 : 256x256x64 persistent ping-pong (row-predicated stores)
  ours-pp-v9 : ping-pong with the store-tolerant stage schedule (padded C rows)
  ours-pp-v12: v9 + bias-armed accumulators (the auto form)
  ours-pp-v13: v12 with non-temporal output stores
  hipblaslt  : torch.nn.functional.linear (bias fused) + the eager activation, the library baseline
The default shapes are the backbone forward as it runs (residual adds live in the LayerNorm
kernel, so out-proj / FFN2 carry bias only); ``--shapes res`` adds the residual-epilogue forms.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import json
import statistics

import torch
import torch.nn.functional as F

from fedrec_with_pytorchdistributed_amd.ops import native


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=78850)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--out", default="")
    ap.add_argument("--only-shape", default="", help="run just this shape name (profiling)")
    ap.add_argument("--only-variants", default="", help="comma list of variant names to keep (profiling)")
    ap.add_argument("--shapes", default="model", help="model | square (8192^3 / 4096^3, no epilogue)")
    a = ap.parse_args()
    lib = native.lib()
    dev = torch.device("cuda")
    shapes = [("qkv", 2304, 768, 0, False), ("out_proj", 768, 768, 0, False), ("ffn1+gelu", 3072, 768, 1, False),
              ("ffn2", 768, 3072, 0, False), ("head_fc1+tanh", 384, 768, 2, False)]
    if a.shapes == "res":
        shapes = [("out_proj+res", 768, 768, 0, True), ("ffn2+res", 768, 3072, 0, True)]
    if a.shapes == "nores":  # the residual shapes without their residual (LN-side residual study)
        shapes = [("out_proj", 768, 768, 0, False), ("out_proj+res", 768, 768, 0, True),
                  ("ffn2", 768, 3072, 0, False), ("ffn2+res", 768, 3072, 0, True)]
    if a.shapes == "square":
        shapes = [("sq8192", 8192, 8192, 0, False), ("sq4096", 4096, 4096, 0, False)]
    if a.only_shape:
        shapes = [s_ for s_ in shapes if s_[0] == a.only_shape]
    res = {}
    for name, N, K, act, has_res in shapes:
        M = N if name.startswith("sq") else a.M
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        b = torch.rand(N, device=dev)
        r = (torch.rand(M, N, device=dev) * 2 - 1).to(torch.bfloat16) if has_res else None
        flops = 2.0 * M * N * K
        variants = {}

        def ours(v):
            def f():
                lib.gemm_set_variant(v)
                return lib.linear(x, w, b, act, r)
            return f

        variants["ours-128"] = ours(0)
        if N % 256 == 0:
            variants["ours-pp-v6"] = ours(6)
            if N <= 3072:
                variants["ours-pp-v9"] = ours(9)
                if not has_res:
                    variants["ours-pp-v12"] = ours(12)
                    variants["ours-pp-v13-nt"] = ours(13)
        elif N % 128 == 0 and N > 256:  # text head N = 384: ping-pong with a partial last column tile
            variants["ours-pp-v9-partial"] = ours(9)
        variants["ours-auto"] = ours(-1)
        bb = b.to(torch.bfloat16)

        def lt():
            y = F.linear(x, w, bb)
            if act == 1:
                y = F.gelu(y)
            elif act == 2:
                y = torch.tanh(y)
            if r is not None:
                y = y + r
            return y

        variants["hipblaslt(+eager epilogue)"] = lt
        if a.only_variants:
            keep = [("hipblaslt(+eager epilogue)" if k == "lib" else k) for k in a.only_variants.split(",")]
            variants = {k: v for k, v in variants.items() if k in keep}
        times = {k: [] for k in variants}
        for f in variants.values():
            f()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for k, f in variants.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    f()
                e.record()
                torch.cuda.synchronize()
                times[k].append(s.elapsed_time(e) / 5)
        lib.gemm_set_variant(-1)
        ref = lt().float()
        row = {}
        for k, ts in times.items():
            med = statistics.median(ts)
            err = float((variants[k]().float() - ref).norm() / ref.norm()) if k.startswith("ours") else float("nan")
            row[k] = {"ms": round(med, 4), "tflops": round(flops / med / 1e9, 1), "rel_err_vs_lib": round(err, 5)}
        res[f"{name} M={M} N={N} K={K}"] = row
        print(name, json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
