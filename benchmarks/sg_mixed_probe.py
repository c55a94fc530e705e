"""Is the text fc's backward launch worth moving onto the LDS-DMA ring?

The launch (HeadFCFn.backward + the user encoder's held-back weight gradients) is mixed-dtype
today: the per-news gradient dnews and the pool's dpre stay fp32 (bias-gradient accuracy), so
it runs on the register-queue mixed kernel.  Splitting each fp32 operand into two bf16 terms
(hi + lo along K, exact to ~2^-16) makes every GEMM bf16 x bf16.  This times both launch forms
at the config-2 shapes (U = 1600 padded titles, 3200 history rows), standalone.

    python benchmarks/sg_mixed_probe.py [out.json]"""
import json
import sys

import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.ops import Gemm


def timeit(fn, iters=50):
    for _ in range(5):
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
U, TD, D, BH, D3, Qd = 1600, 768, 400, 3200, 1200, 200
dnews = torch.randn(U, D, device=dev)
fcb = (torch.randn(D, TD, device=dev) * 0.05).to(bf)  # [K = D, N = TD] (b_mode 1)
pooled = torch.randn(U, TD, device=dev).to(bf)
dqkv = torch.randn(BH, D3, device=dev).to(bf)
xb = torch.randn(BH, D, device=dev).to(bf)
dpre = torch.randn(BH, Qd, device=dev)
c3b = torch.randn(BH, D, device=dev).to(bf)


def hi_lo(x):
    hi = x.to(bf)
    return hi, (x - hi.float()).to(bf)


out = {}
c_dp = torch.empty(U, TD, device=dev)
c_fw = torch.empty(D, TD, device=dev)
c_q = torch.empty(D3, D, device=dev)
c_w1 = torch.empty(Qd, D, device=dev)
s_fw, s_q, s_w1 = (torch.empty(n, device=dev) for n in (D, D3, Qd))
mixed = [Gemm(dnews, fcb, c_dp, U, TD, D, D, TD, TD, b_mode=1),
         Gemm(dnews, pooled, c_fw, D, TD, U, D, TD, TD, a_mode=1, b_mode=1, asum=s_fw),
         Gemm(dqkv, xb, c_q, D3, D, BH, D3, D, D, a_mode=1, b_mode=1, asum=s_q),
         Gemm(dpre, c3b, c_w1, Qd, D, BH, Qd, D, D, a_mode=1, b_mode=1, asum=s_w1)]
out["mixed_launch_us"] = timeit(lambda: ops.small_gemm(*mixed))

# hi / lo operands: dnews [U, 2D] (hi | lo along K) against [fc; fc]; dnews rows stacked (K = 2U)
# against pooled stacked; dpre rows stacked (K = 2 BH) against c3b stacked
dh, dl = hi_lo(dnews)
dn2 = torch.cat([dh, dl], 1).contiguous()
fc2 = torch.cat([fcb, fcb], 0).contiguous()
dnr = torch.cat([dh, dl], 0).contiguous()
pool2 = torch.cat([pooled, pooled], 0).contiguous()
ph, pl = hi_lo(dpre)
dpr = torch.cat([ph, pl], 0).contiguous()
c3r = torch.cat([c3b, c3b], 0).contiguous()
allbf = [Gemm(dn2, fc2, c_dp, U, TD, 2 * D, 2 * D, TD, TD, b_mode=1),
         Gemm(dnr, pool2, c_fw, D, TD, 2 * U, D, TD, TD, a_mode=1, b_mode=1, asum=s_fw),
         Gemm(dqkv, xb, c_q, D3, D, BH, D3, D, D, a_mode=1, b_mode=1, asum=s_q),
         Gemm(dpr, c3r, c_w1, Qd, D, 2 * BH, Qd, D, D, a_mode=1, b_mode=1, asum=s_w1)]
out["bf16_hilo_launch_us"] = timeit(lambda: ops.small_gemm(*allbf))
# accuracy of the hi / lo form against fp32 (the fc dgrad and the two weight gradients)
ops.small_gemm(*allbf)
torch.cuda.synchronize()
ref_dp = dnews @ fcb.float()
ref_w1 = dpre.t() @ c3b.float()
out["fc_dgrad_rel_err"] = float((c_dp - ref_dp).norm() / ref_dp.norm())
out["w1_grad_rel_err"] = float((c_w1 - ref_w1).norm() / ref_w1.norm())
out["w1_bias_rel_err"] = float((s_w1 - dpre.sum(0)).norm() / dpre.sum(0).norm())
for k, v in out.items():
    out[k] = round(v, 3) if k.endswith("_us") else v
print(json.dumps(out), flush=True)
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
