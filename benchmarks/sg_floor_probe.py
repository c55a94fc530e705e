"""Where the fixed time of a small-GEMM launch goes: device durations (run under rocprofv3
--kernel-trace) of launches whose work shrinks to nothing -- one block, one k-step, full grid at
one k-step, the config-2 att_fc1 shape -- for the LDS-DMA form (tile 0) and the register-direct
form (1003).  Each launch runs alone (synchronised), so the trace's begin -> end is the kernel.

    rocprofv3 --kernel-trace --output-format csv -d out -o p -- python benchmarks/sg_floor_probe.py
"""
import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.ops import Gemm, native

dev = torch.device("cuda", 0)
bf = torch.bfloat16
native.lib()
shapes = [(64, 64, 32), (64, 64, 400), (3200, 200, 32), (3200, 200, 400), (3200, 1200, 32), (3200, 1200, 400)]
for M, N, K in shapes:
    A = torch.randn(M, K, device=dev).to(bf)
    B = torch.randn(N, K, device=dev).to(bf)
    C = torch.empty(M, N, device=dev)
    for tile in (0, 1003):
        g = Gemm(A, B, C, M, N, K, K, K, N)
        for _ in range(12):
            ops.small_gemm(g, tile=tile)
            torch.cuda.synchronize()
        print(M, N, K, tile, flush=True)
x = torch.empty(3200 * 200, device=dev)
for _ in range(12):
    x.fill_(1.0)  # a trivial 1-pass kernel for the launch floor
    torch.cuda.synchronize()
