import torch
from fedrec_with_pytorchdistributed_amd.parallel.ipc_allreduce import LocalIpcGroup
dev = torch.device("cuda", 0)
for mode in ("one", "two", "two"):
    g = LocalIpcGroup(2, dev, cap=1 << 20, blocks=8)
    for n in (4, 8, 1024):
        xs = [torch.arange(n, device=dev, dtype=torch.float32) + 100 * r for r in range(2)]
        exp = xs[0] + xs[1]
        g.allreduce_(xs, mode)
        torch.cuda.synchronize()
        print(mode, n, "status", g.status(), "ok", [bool(torch.equal(x, exp)) for x in xs], xs[0][:4].tolist(), xs[1][:4].tolist(), flush=True)
    g.close()
