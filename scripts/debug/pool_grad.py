import os, sys
sys.path.insert(0, os.getcwd())
import torch
from fedrec_with_pytorchdistributed_amd.ops import functional as OF
torch.manual_seed(0)
n, T, D, Q = 16, 50, 400, 200
x = torch.randn(n, T, D)
lin1 = torch.nn.Linear(D, Q); lin2 = torch.nn.Linear(Q, 1)
g = torch.randn(n, D)
def run(dev):
    l1 = torch.nn.Linear(D, Q).to(dev); l2 = torch.nn.Linear(Q, 1).to(dev)
    l1.load_state_dict(lin1.state_dict()); l2.load_state_dict(lin2.state_dict())
    xx = x.clone().to(dev).detach().requires_grad_(True)
    out = OF.additive_pool(xx, l1, l2)
    out.backward(g.to(dev))
    gs = [xx.grad, l1.weight.grad, l1.bias.grad, l2.weight.grad]
    print(dev, [None if t is None else t.shape for t in gs])
    return [out.detach().cpu()] + [torch.zeros(1) if t is None else t.cpu() for t in gs]
a = run(torch.device("cpu")); b = run(torch.device("cuda"))
for name, u, v in zip(["out", "dx", "dW1", "db1", "dw2"], a, b):
    print(name, float((u - v).norm() / (u.norm() + 1e-12)), float(u.norm()), float(v.norm()))
