"""The user step's small GEMMs (csrc/small_gemm.hip) at the config-2 shapes, every tile variant,
fp32 vs bf16 operands, separate vs concatenated Q|K|V weights; plus the bias-gradient colsum
and the bf16 wgrad kernel (gemm_wgrad.hip) on the concatenated dW_qkv for comparison.

    python benchmarks/small_gemm_bench.py [--BH 3200] [--U 1664] [--iters 40]

One JSON line per (case, tile): us per launch (launch + split-K reduce), and the max relative
error against the bf16-rounded fp32 emulation (ops.small_gemm_ref) so a fast wrong variant
cannot pass unnoticed."""
import argparse
import json

import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.ops import Gemm, native


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


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--BH", type=int, default=3200)
    ap.add_argument("--U", type=int, default=1664)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    BH, D, Qd, U, KT = a.BH, 400, 200, a.U, 768
    r = lambda *s: torch.randn(*s, device=dev)  # noqa: E731
    xd = r(BH, D)
    xdh = xd.to(torch.bfloat16)
    wq, wk, wv, w1 = r(D, D) * .05, r(D, D) * .05, r(D, D) * .05, r(Qd, D) * .05
    wcat = torch.cat([wq, wk, wv])
    wcath = wcat.to(torch.bfloat16)
    bcat = r(3 * D)
    qkv = torch.zeros(BH, 3 * D, device=dev)
    c3, e = r(BH, D), torch.zeros(BH, Qd, device=dev)
    dpre, dctx = r(BH, Qd), r(BH, D)
    dqkv = r(BH, 3 * D)
    dqkvh = dqkv.to(torch.bfloat16)
    dx = torch.zeros(BH, D, device=dev)
    gcat, gw1 = torch.zeros(3 * D, D, device=dev), torch.zeros(Qd, D, device=dev)
    xt, wt, bt = r(U, KT), r(D, KT) * .05, r(D)
    yt, dyt = torch.zeros(U, D, device=dev), r(U, D)
    dxt, dwt = torch.zeros(U, KT, device=dev), torch.zeros(D, KT, device=dev)

    cases = {
        "qkv_3x400_f32": lambda: [Gemm(xd, w, qkv[:, s * D:(s + 1) * D], BH, D, D, D, D, 3 * D, bias=bcat[s * D:])
                                  for s, w in enumerate((wq, wk, wv))],
        "qkv_cat_f32": lambda: [Gemm(xd, wcat, qkv, BH, 3 * D, D, D, D, 3 * D, bias=bcat)],
        "qkv_cat_bf16": lambda: [Gemm(xdh, wcath, qkv, BH, 3 * D, D, D, D, 3 * D, bias=bcat)],
        "fc1_f32": lambda: [Gemm(c3, w1, e, BH, Qd, D, D, D, Qd, bias=bcat[:Qd], act=1)],
        "dctx_f32": lambda: [Gemm(dpre, w1, dctx, BH, D, Qd, Qd, D, D, b_mode=1, accumulate=True)],
        "dgrad_kseg_f32": lambda: [Gemm(dqkv, wq, dx, BH, D, 3 * D, 3 * D, D, D, b_mode=1, bseg=(wk, wv), kseg=D)],
        "dgrad_cat_bf16B": lambda: [Gemm(dqkv, wcath, dx, BH, D, 3 * D, 3 * D, D, D, b_mode=1)],
        "dgrad_cat_bf16AB": lambda: [Gemm(dqkvh, wcath, dx, BH, D, 3 * D, 3 * D, D, D, b_mode=1)],
        "wgrad_4_f32": lambda: [Gemm(dqkv[:, s * D:(s + 1) * D], xd, gcat[s * D:(s + 1) * D], D, D, BH, 3 * D, D, D,
                                     a_mode=1, b_mode=1) for s in range(3)]
        + [Gemm(dpre, c3, gw1, Qd, D, BH, Qd, D, D, a_mode=1, b_mode=1)],
        "wgrad_cat_f32": lambda: [Gemm(dqkv, xd, gcat, 3 * D, D, BH, 3 * D, D, D, a_mode=1, b_mode=1),
                                  Gemm(dpre, c3, gw1, Qd, D, BH, Qd, D, D, a_mode=1, b_mode=1)],
        "wgrad_cat_bf16B": lambda: [Gemm(dqkv, xdh, gcat, 3 * D, D, BH, 3 * D, D, D, a_mode=1, b_mode=1),
                                    Gemm(dpre, c3, gw1, Qd, D, BH, Qd, D, D, a_mode=1, b_mode=1)],
        "wgrad_cat_bf16AB": lambda: [Gemm(dqkvh, xdh, gcat, 3 * D, D, BH, 3 * D, D, D, a_mode=1, b_mode=1),
                                     Gemm(dpre, c3, gw1, Qd, D, BH, Qd, D, D, a_mode=1, b_mode=1)],
        "wgrad_3+1_bf16B_mixed": lambda: [Gemm(dqkv[:, s * D:(s + 1) * D], xdh, gcat[s * D:(s + 1) * D], D, D, BH,
                                               3 * D, D, D, a_mode=1, b_mode=1) for s in range(3)]
        + [Gemm(dpre, c3, gw1, Qd, D, BH, Qd, D, D, a_mode=1, b_mode=1)],
        "fc1_bf16B": lambda: [Gemm(c3, wcath[:Qd], e, BH, Qd, D, D, D, Qd, bias=bcat[:Qd], act=1)],
        "dctx_bf16B": lambda: [Gemm(dpre, wcath[:Qd], dctx, BH, D, Qd, Qd, D, D, b_mode=1, accumulate=True)],
        "dgrad_cat_bf16B_drop": lambda: [Gemm(dqkv, wcath, dx, BH, D, 3 * D, 3 * D, D, D, b_mode=1, pdrop=0.2, drop_on=3,
                                              drop_ld=D, seed=1, offset=2)],
        "textfc_fwd_f32": lambda: [Gemm(xt, wt, yt, U, D, KT, KT, KT, D, bias=bt)],
        "textfc_bwd_f32": lambda: [Gemm(dyt, wt, dxt, U, KT, D, D, KT, KT, b_mode=1),
                                   Gemm(dyt, xt, dwt, D, KT, U, D, KT, KT, a_mode=1, b_mode=1)],
    }
    out = []
    for name, mk in cases.items():
        for tile in (0, 1, 2, 3, 4):
            gs = mk()
            snap = [g.C.clone() for g in gs]
            wants = [ops.small_gemm_ref(g) for g in gs]
            ops.small_gemm(*gs, tile=tile)
            torch.cuda.synchronize()
            err = max(rel(torch.as_strided(g.C, (g.M, g.N), (g.ldc, 1)), w) for g, w in zip(gs, wants))
            for g, s0 in zip(gs, snap):
                g.C.copy_(s0)
            us = timeit(lambda: ops.small_gemm(*gs, tile=tile), a.iters)
            flops = sum(2.0 * g.M * g.N * g.K for g in gs)
            rec = {"case": name, "tile": tile, "us": round(us, 2), "TF": round(flops / us / 1e6, 1), "rel_err": err}
            out.append(rec)
            print(json.dumps(rec), flush=True)
    lib = native.lib()
    us = timeit(lambda: lib.wgrad(dqkvh, xdh), a.iters)
    rec = {"case": "wgrad_kernel_bf16_dWqkv", "us": round(us, 2)}
    out.append(rec)
    print(json.dumps(rec), flush=True)
    gb = [torch.zeros(n, device=dev) for n in (D, D, D, Qd)]
    us = timeit(lambda: ops.colsum_f32([(dqkv[:, 0:D], gb[0], BH, D, 3 * D), (dqkv[:, D:2 * D], gb[1], BH, D, 3 * D),
                                        (dqkv[:, 2 * D:], gb[2], BH, D, 3 * D), (dpre, gb[3], BH, Qd, Qd)]), a.iters)
    rec = {"case": "colsum_user_bias_grads", "us": round(us, 2)}
    out.append(rec)
    print(json.dumps(rec), flush=True)
    us = timeit(lambda: ops.gather_dropout(c3, torch.arange(BH, device=dev, dtype=torch.int32), 0.2, 1, 2), a.iters)
    print(json.dumps({"case": "gather_dropout_f32", "us": round(us, 2)}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
