"""Register-direct small GEMM (``small_gemm_rd_kernel``) against the default launch form on the
config-2 step's bf16 x bf16 shapes, timed inside a captured HIP graph (device time per launch
incl. the inter-kernel gap, as the step graph sees it -- eager timing of these launches is
host-bound), and checked against the fp32 emulation ``ops.small_gemm_ref``.

    python benchmarks/sg_rd_bench.py [out.jsonl]
"""
import json
import sys

import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.ops import Gemm, native

dev = torch.device("cuda", 0)
bf = torch.bfloat16
torch.manual_seed(0)
native.lib()
out = open(sys.argv[1], "w") if len(sys.argv) > 1 else None


def graph_us(fn, reps=20, replays=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(replays):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1e3 / (reps * replays)


BH, D, D3, Qd, U, TD = 3200, 400, 1200, 200, 1600, 768
x_b = torch.randn(BH, D, device=dev).to(bf)
wqkv_b = (torch.randn(D3 + Qd, D, device=dev) * 0.05).to(bf)
w1t_b = wqkv_b[D3:].t().contiguous()
wqkvt_b = wqkv_b[:D3].t().contiguous()
dpre_b = torch.randn(BH, Qd, device=dev).to(bf)
dqkv_b = torch.randn(BH, D3, device=dev).to(bf)
pooled_b = torch.randn(U, TD, device=dev).to(bf)
fc_b = (torch.randn(D, TD, device=dev) * 0.05).to(bf)
fct_b = fc_b.t().contiguous()
dnews_b = torch.randn(U, D, device=dev).to(bf)
bias3 = torch.randn(D3, device=dev)
bias1 = torch.randn(Qd, device=dev)
biasf = torch.randn(D, device=dev)

shapes = {
    "text_fc_fwd": lambda: Gemm(pooled_b, fc_b, torch.empty(U, D, device=dev), U, D, TD, TD, TD, D, bias=biasf),
    "qkv_fwd": lambda: Gemm(x_b, wqkv_b[:D3], torch.empty(BH, D3, device=dev), BH, D3, D, D, D, D3, bias=bias3),
    "att_fc1_fwd": lambda: Gemm(x_b, wqkv_b[D3:], torch.empty(BH, Qd, device=dev), BH, Qd, D, D, D, Qd, bias=bias1,
                                act=1),
    "dctx_nt": lambda: Gemm(dpre_b, w1t_b, torch.randn(BH, D, device=dev), BH, D, Qd, Qd, Qd, D, accumulate=True),
    "dgrad_nt_drop": lambda: Gemm(dqkv_b, wqkvt_b, torch.empty(BH, D, device=dev), BH, D, D3, D3, D3, D, pdrop=0.2,
                                  drop_on=3, drop_ld=D, seed=7, offset=3),
    "fc_dgrad_nt": lambda: Gemm(dnews_b, fct_b, torch.empty(U, TD, device=dev), U, TD, D, D, D, TD),
}
variants = [0, 1002, 1003, 1004, 1012, 1013, 1022, 1023, 1032, 1033, 1103, 1113]
for name, mk in shapes.items():
    g = mk()
    c0 = g.C.clone()
    refc = ops.small_gemm_ref(g)
    for v in variants:
        g.C.copy_(c0)
        try:
            ops.small_gemm(g, tile=v)
        except RuntimeError as e:
            print(name, v, "rejected", str(e)[:80], flush=True)
            continue
        torch.cuda.synchronize()
        err = ((g.C - refc).abs().max() / refc.abs().max().clamp_min(1e-30)).item()
        us = graph_us(lambda: ops.small_gemm(g, tile=v))
        rec = {"gemm": name, "tile": v, "us": round(us, 2), "rel_err": float(f"{err:.3g}"),
               "TF": round(2.0 * g.M * g.N * g.K / us / 1e6, 1)}
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
