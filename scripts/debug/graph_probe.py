"""Probe which part of a step breaks HIP-graph capture (debug helper)."""
import os, sys, traceback
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

dev = torch.device("cuda", 0)


def cap(name, fn, warm=True):
    try:
        if warm:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = fn()
        g.replay()
        torch.cuda.synchronize()
        print("OK  ", name, flush=True)
        return g, out
    except Exception as e:
        print("FAIL", name, type(e).__name__, str(e)[:200], flush=True)
        return None, None


x = torch.randn(1024, 1024, device=dev)
cap("matmul", lambda: x @ x)
cap("matmul nowarm", lambda: x @ x, warm=False)
w = torch.randn(64, 64, device=dev, requires_grad=True)
def fb():
    w.grad = None
    y = (torch.randn(8, 64, device=dev) @ w).sum()
    y.backward()
    return y
cap("autograd", fb)
from fedrec_with_pytorchdistributed_amd.ops import native
native.lib()
from fedrec_with_pytorchdistributed_amd import ops
a = torch.randn(512, 768, device=dev).to(torch.bfloat16)
wt = torch.randn(384, 768, device=dev).to(torch.bfloat16)
cap("fedrec.linear", lambda: ops.linear(a, wt, None, act="tanh"))
r = torch.randn(100, 400, device=dev)
inv = torch.randint(0, 10, (100,), device=dev, dtype=torch.int32)
perm, ptr = ops.segments_from_inv(inv, 10)
cap("segment_sum", lambda: ops.segment_sum_rows(r, inv, 10, seg=(perm, ptr)))
cap("dropout torch", lambda: torch.nn.functional.dropout(r, 0.2, True))
