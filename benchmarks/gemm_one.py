"""Run one GEMM shape/variant repeatedly (for rocprofv3 counter collection)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fedrec_with_pytorchdistributed_amd.ops import native

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=78850)
ap.add_argument("--N", type=int, default=2304)
ap.add_argument("--K", type=int, default=768)
ap.add_argument("--act", type=int, default=0)
ap.add_argument("--variant", type=int, default=2)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--lib", action="store_true")
a = ap.parse_args()
lib = native.lib()
dev = torch.device("cuda")
x = (torch.rand(a.M, a.K, device=dev) * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(a.N, a.K, device=dev) * 2 - 1) / a.K ** 0.5).to(torch.bfloat16)
b = torch.rand(a.N, device=dev)
lib.gemm_set_variant(a.variant)
for _ in range(a.iters):
    if a.lib:
        torch.nn.functional.linear(x, w, b.to(torch.bfloat16))
    else:
        lib.linear(x, w, b, a.act, None)
torch.cuda.synchronize()
print("done")
