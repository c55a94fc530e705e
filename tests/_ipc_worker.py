"""Multi-process worker for test_ipc_allreduce_multiprocess: W processes on ONE GPU (same-device
IPC), gloo control group, the IPC all-reduce against gloo's all-reduce of the same data."""
import sys

import torch
import torch.distributed as dist

from fedrec_with_pytorchdistributed_amd.parallel.ipc_allreduce import IpcAllReduce

dist.init_process_group("gloo")
rank, W = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
try:
    g = IpcAllReduce(None, rank, W, dev, cap=4 << 20, one_shot_max=1 << 20, blocks=8)
except Exception as e:  # the runtime refused same-device IPC: reported, not a failure of the protocol
    print(f"IPC_UNAVAILABLE {e!r}", flush=True)
    dist.destroy_process_group()
    sys.exit(0)
ok = True
for step, (n, dt) in enumerate([(4, torch.float32), (1000, torch.float32), (1 << 18, torch.float32),
                                (3 << 18, torch.float32), (5 << 20, torch.float32), (777, torch.int32),
                                (1 << 20, torch.int32)]):
    gen = torch.Generator().manual_seed(1000 * step + rank)
    if dt == torch.float32:
        x = torch.randn(n, generator=gen)
    else:
        x = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), generator=gen, dtype=torch.int64).to(torch.int32)
    ref = x.clone().to(torch.int64) if dt == torch.int32 else x.clone().double()
    dist.all_reduce(ref)
    y = x.to(dev)
    g.allreduce_(y)
    torch.cuda.synchronize()
    got = y.cpu()
    if dt == torch.int32:
        exp = ((ref + (1 << 31)) % (1 << 32) - (1 << 31)).to(torch.int32)  # wrap-around sum
        good = torch.equal(got, exp)
    else:
        good = torch.allclose(got.double(), ref, rtol=1e-6, atol=1e-5)
    if not good:
        ok = False
        print(f"MISMATCH n={n} dtype={dt}", flush=True)
    # every rank must hold the bitwise-same result
    allg = [torch.zeros_like(got) for _ in range(W)]
    dist.all_gather(allg, got)
    if not all(torch.equal(allg[0], a) for a in allg):
        ok = False
        print(f"RANKS DIFFER n={n}", flush=True)
st = g.status()
g.close()
print("IPC OK" if ok and st == 0 else f"IPC FAIL status={st}", flush=True)
dist.destroy_process_group()
