"""Backward-GEMM microbenchmark at the BERT-base training shapes (config 5, M = tokens/step).

dgrad  dX[M, Kin] = dY[M, Nout] @ W[Nout, Kin] (+ residual)
  lib   : torch.mm / addmm_ (hipBLASLt, NN)
  ours  : our NT ping-pong GEMM on the pre-transposed weight W^T [Kin, Nout] (the transpose
          is a per-step 1-5 MB copy, timed separately as ``wT``)
wgrad  dW[Nout, Kin] = dY^T X
  lib   : the library form of ops.functional.wgrad (split-K bmm + sum)
  ours  : our TN MFMA kernel (csrc/gemm_wgrad.hip)

All variants interleaved in one process, median of ``--rounds`` per variant.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedrec_with_pytorchdistributed_amd.ops import native  # noqa: E402
from fedrec_with_pytorchdistributed_amd.ops import functional as OF  # noqa: E402


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=78260)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    lib = native.lib()
    dev = torch.device("cuda")
    M = a.M
    # (name, Nout, Kin, residual)
    shapes = [("qkv", 2304, 768, True), ("out_proj", 768, 768, False), ("ffn1", 3072, 768, True),
              ("ffn2", 768, 3072, False), ("head_fc1", 384, 768, False)]
    g = torch.Generator(device=dev).manual_seed(0)
    rows = []
    for name, N, K, res in shapes:
        dy = (torch.randn(M, N, device=dev, generator=g) * 0.1).bfloat16()
        x = (torch.randn(M, K, device=dev, generator=g) * 0.1).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).bfloat16()
        r = (torch.randn(M, K, device=dev, generator=g) * 0.1).bfloat16() if res else None
        wT = w.t().contiguous()
        ref = (dy.float() @ w.float() + (r.float() if res else 0)).bfloat16()
        out = lib.linear(dy, wT, None, 0, r)
        err = float((out.float() - ref.float()).abs().max() / ref.float().abs().max())
        v = {"lib": [], "ours": [], "wT": [], "wgrad_lib": [], "wgrad_ours": []}
        wref = dy.float().t() @ x.float()
        wo = lib.wgrad(dy, x)
        row_err = float((wo - wref).abs().max() / wref.abs().max())

        def wg(impl):
            OF._WGRAD_IMPL = impl
            return OF.wgrad(dy, x)

        def lib_fn():
            if res:
                r2 = r.clone()
                return r2.addmm_(dy, w)
            return torch.mm(dy, w)

        for _ in range(a.rounds):
            v["lib"].append(timeit(lib_fn))
            v["ours"].append(timeit(lambda: lib.linear(dy, wT, None, 0, r)))
            v["wT"].append(timeit(lambda: w.t().contiguous()))
            v["wgrad_lib"].append(timeit(lambda: wg("lib")))
            v["wgrad_ours"].append(timeit(lambda: wg("ours")))
        flop = 2.0 * M * N * K
        row = {"shape": name, "M": M, "N_out": N, "K_in": K, "residual": res, "rel_err": err, "wgrad_rel_err": row_err}
        for k, t in v.items():
            ms = statistics.median(t)
            row[f"{k}_us"] = round(ms * 1e3, 1)
            if k != "wT":
                row[f"{k}_TF"] = round(flop / ms / 1e9, 1)
        print(json.dumps(row), flush=True)
        rows.append(row)
    return 0


if __name__ == "__main__":
    sys.exit(main())
