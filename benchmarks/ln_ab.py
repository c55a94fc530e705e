import sys, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/benchmarks")
from kernel_bench import timeit
from fedrec_with_pytorchdistributed_amd.ops import native
lib = native.lib(); dev = torch.device("cuda")
M, D = 78850, 768
x = torch.randn(M, D, device=dev).to(torch.bfloat16); r = torch.randn(M, D, device=dev).to(torch.bfloat16)
w, b = torch.randn(D, device=dev), torch.randn(D, device=dev)
for rep in range(3):
    for wide in (1, 4, 2, 3, 0):
        lib.ln_set_wide(wide)
        ms_r = timeit(lambda: lib.layer_norm(x, w, b, 1e-12, r), iters=50)
        ms = timeit(lambda: lib.layer_norm(x, w, b, 1e-12), iters=50)
        print(rep, wide, "res", round(ms_r * 1000, 1), "us", round(3 * M * D * 2 / ms_r / 1e6), "GB/s | plain", round(ms * 1000, 1), "us", flush=True)
