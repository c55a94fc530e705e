"""Time each small GEMM of the config-2 step standalone, in the operand forms the step uses and
in candidate forms (bf16 operands, DMA-ring stage counts): which launches are worth moving.

    python benchmarks/sg_step_shapes.py [out.json]

Shapes (B = 64 impressions, H = 50 history, D = 400, Qd = 200, U ~ 1565 titles, text D 768):
user Q|K|V fwd 3200x1200x400, att_fc1 fwd 3200x200x400, dctx += dpre W1 3200x400x200 (B
stored transposed), dgrad 3200x400x1200 (B transposed), wgrads [1200|200]x400 over K = 3200
(both transposed), text fc fwd 1565x400x768, fc dgrad 1565x768x400, fc wgrad 400x768 over 1565."""
import json
import sys

import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.ops import Gemm


def timeit(fn, iters=40):
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


dev = torch.device("cuda", 0)
bf = torch.bfloat16
torch.manual_seed(0)
out = []


def run(name, make, tiles=(0, 5, 6, 9)):
    for dt in ("f32", "bf16"):
        gs = make(dt)
        if gs is None:
            continue
        for t in tiles:
            us = timeit(lambda: ops.small_gemm(*gs, tile=t))
            rec = {"gemm": name, "operands": dt, "tile": t, "us": round(us, 2)}
            out.append(rec)
            print(json.dumps(rec), flush=True)


def cvt(x, dt):
    return x.to(bf) if dt == "bf16" else x


BH, D, D3, Qd, U, TD = 3200, 400, 1200, 200, 1600, 768  # U: the step graph pads the unique titles
x_b = torch.randn(BH, D, device=dev).to(bf)
wqkv_b = (torch.randn(D3 + Qd, D, device=dev) * 0.05).to(bf)
w1t_b = wqkv_b[D3:].t().contiguous()  # [D, Qd]
wqkvt_b = wqkv_b[:D3].t().contiguous()  # [D, D3]
c3 = torch.randn(BH, D, device=dev)
dpre = torch.randn(BH, Qd, device=dev)
dqkv = torch.randn(BH, D3, device=dev)
pooled_b = torch.randn(U, TD, device=dev).to(bf)
fc_b = (torch.randn(D, TD, device=dev) * 0.05).to(bf)
fct_b = fc_b.t().contiguous()
dnews = torch.randn(U, D, device=dev)

run("qkv_fwd", lambda dt: [Gemm(x_b, wqkv_b[:D3], torch.empty(BH, D3, device=dev), BH, D3, D, D, D, D3)]
    if dt == "bf16" else None)
run("att_fc1_fwd", lambda dt: [Gemm(cvt(c3, dt), wqkv_b[D3:], torch.empty(BH, Qd, device=dev), BH, Qd, D, D, D, Qd,
                                    act=1)])
run("dctx_nn", lambda dt: [Gemm(cvt(dpre, dt), wqkv_b[D3:], torch.zeros(BH, D, device=dev), BH, D, Qd, Qd, D, D,
                                b_mode=1, accumulate=True)])
run("dctx_nt_on_w1t", lambda dt: [Gemm(cvt(dpre, dt), w1t_b, torch.zeros(BH, D, device=dev), BH, D, Qd, Qd, Qd, D,
                                       accumulate=True)])
run("dgrad_nn", lambda dt: [Gemm(cvt(dqkv, dt), wqkv_b[:D3], torch.empty(BH, D, device=dev), BH, D, D3, D3, D, D,
                                 b_mode=1)])
run("dgrad_nt_on_wt", lambda dt: [Gemm(cvt(dqkv, dt), wqkvt_b, torch.empty(BH, D, device=dev), BH, D, D3, D3, D3, D)])
run("wgrads_tn", lambda dt: [Gemm(cvt(dqkv, dt), x_b, torch.empty(D3, D, device=dev), D3, D, BH, D3, D, D, a_mode=1,
                                  b_mode=1, asum=torch.empty(D3, device=dev)),
                             Gemm(cvt(dpre, dt), cvt(c3, dt), torch.empty(Qd, D, device=dev), Qd, D, BH, Qd, D, D,
                                  a_mode=1, b_mode=1, asum=torch.empty(Qd, device=dev))], tiles=(0, 9))
# the user backward's weight-gradient launch as the step issues it (dgrad + Q|K|V weight gradient
# on bf16 dQ|dK|dV, dW1 on the fp32 dpre: the mixed kernel) and its all-bf16 part alone
dqkv_b, c3b = dqkv.to(bf), c3.to(bf)
da8 = torch.randn(BH, 8, device=dev)
e3 = torch.randn(BH, Qd, device=dev)
run("user_wg_launch", lambda dt: [Gemm(dqkv_b, wqkv_b[:D3], torch.empty(BH, D, device=dev), BH, D, D3, D3, D, D, b_mode=1),
                                  Gemm(dqkv_b, x_b, torch.empty(D3, D, device=dev), D3, D, BH, D3, D, D, a_mode=1,
                                       b_mode=1, asum=torch.empty(D3, device=dev)),
                                  Gemm(dpre, c3b, torch.empty(Qd, D, device=dev), Qd, D, BH, Qd, D, D, a_mode=1,
                                       b_mode=1, asum=torch.empty(Qd, device=dev)),
                                  Gemm(da8, e3, torch.empty(8, Qd, device=dev), 8, Qd, BH, 8, Qd, Qd, a_mode=1, b_mode=1,
                                       asum=torch.empty(8, device=dev))] if dt == "bf16" else None, tiles=(0,))
run("user_wg_bf16_part", lambda dt: [Gemm(dqkv_b, wqkv_b[:D3], torch.empty(BH, D, device=dev), BH, D, D3, D3, D, D,
                                          b_mode=1),
                                     Gemm(dqkv_b, x_b, torch.empty(D3, D, device=dev), D3, D, BH, D3, D, D, a_mode=1,
                                          b_mode=1, asum=torch.empty(D3, device=dev))] if dt == "bf16" else None,
    tiles=(0, 9))
run("fc_fwd", lambda dt: [Gemm(pooled_b, fc_b, torch.empty(U, D, device=dev), U, D, TD, TD, TD, D)]
    if dt == "bf16" else None)
run("fc_dgrad_nn", lambda dt: [Gemm(cvt(dnews, dt), fc_b, torch.empty(U, TD, device=dev), U, TD, D, D, TD, TD,
                                    b_mode=1)])
run("fc_dgrad_nt_on_fct", lambda dt: [Gemm(cvt(dnews, dt), fct_b, torch.empty(U, TD, device=dev), U, TD, D, D, D, TD)])
run("fc_wgrad_tn", lambda dt: [Gemm(cvt(dnews, dt), pooled_b, torch.empty(D, TD, device=dev), D, TD, U, D, TD, TD,
                                    a_mode=1, b_mode=1, asum=torch.empty(D, device=dev))], tiles=(0,))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
