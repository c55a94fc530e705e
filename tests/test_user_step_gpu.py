"""The fused device user side (ops.functional.UserStepFn: our GEMMs + kernels end to end)
against the fp32 CPU oracle of the reference math (UserEncoder modules + score_ce) under the
same Philox input-dropout mask: loss, scores, the per-news gradient and every user-encoder
parameter gradient; plus the text head's FC on the small GEMM."""
import copy

import pytest
import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.config import FedRecConfig
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
from fedrec_with_pytorchdistributed_amd.ops import functional as OF
from fedrec_with_pytorchdistributed_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _his_ids(B, H, dev):
    """History ids with padded slots (0): impression b keeps its first H - 6 b slots, the
    last impression none (a fully masked row)."""
    ids = torch.randint(1, 300, (B, H), dtype=torch.int32)
    for b in range(B):
        ids[b, max(0, H - 6 * b):] = 0
    ids[-1] = 0
    return ids.to(dev)


@pytest.mark.parametrize("p,mask", [(0.0, False), (0.2, False), (0.2, True)])
def test_user_step_matches_module_oracle(dev, p, mask):
    """``mask``: the mask_padding option -- the padded history slots are masked keys of the
    attention and masked positions of the pool (kernels vs the host oracle's masked softmax)."""
    torch.manual_seed(0)
    cfg = FedRecConfig(mode="grad_avg", mask_padding=mask)
    model = FedRecModel(cfg)
    ue_c = model.user_encoder
    ue_g = copy.deepcopy(ue_c).to(dev)
    D, B, C, H = 400, 8, 5, 50
    ids = torch.randint(0, 300, (B * (C + H),), dtype=torch.int32, device=dev)
    uniq, inv, perm, ptr = ops.dedup(ids, 300)  # the engine's layout: every row of v has occurrences
    U = uniq.numel()
    v = (torch.randn(U, D) * 0.05).to(dev).requires_grad_(True)
    seed, off, step = 1234, 7, 3
    rng = torch.tensor([step], dtype=torch.int64, device=dev)
    his_ids = _his_ids(B, H, dev) if mask else None
    loss, scores = OF.user_step(v, inv, perm, ptr, ue_g, B, C, H, "sigmoid", (p, seed, off), rng, (0.0, 0.0, 0, 0),
                                False, his_ids)
    loss.backward()
    # oracle: fp32 CPU, the same gathered rows and the same mask (offset off + step)
    vc = v.detach().cpu().requires_grad_(True)
    rows = vc[inv.long().cpu()]
    cand, his = rows[: B * C].view(B, C, D), rows[B * C:]
    if p > 0:
        idx = torch.arange(B * H)[:, None] * D + torch.arange(D)[None, :]
        his = his * R.dropout_scale(idx, p, seed, off + step)
    ue_c.eval()  # the mask is applied above; the module's own dropout stays off
    u = ue_c(his.view(B, H, D), None if his_ids is None else his_ids.cpu())
    loss_c, s_c, _, _ = R.score_ce_fwd_bwd(cand, u, "sigmoid")
    # score_ce_fwd_bwd returns analytic grads; recompute the loss under autograd for the backward
    sc = torch.sigmoid(torch.bmm(cand, u.unsqueeze(-1)).squeeze(-1))
    lc = torch.nn.functional.cross_entropy(sc, torch.zeros(B, dtype=torch.long))
    lc.backward()
    assert abs(float(loss) - float(lc)) < 2e-4, (float(loss), float(lc))
    assert float((scores.cpu() - sc.detach()).abs().max()) < 2e-3
    assert _rel(v.grad, vc.grad) < 3e-2, _rel(v.grad, vc.grad)
    for (n, pg), (_, pc) in zip(ue_g.named_parameters(), ue_c.named_parameters()):
        if float(pc.grad.norm()) < 1e-8:
            # rounding noise: the key bias (softmax shift invariance) and, at random init, the
            # user pool (its inputs are nearly identical rows, so d alpha cancels): ~1e-11
            assert float(pg.grad.norm()) < 1e-6, n
            continue
        assert _rel(pg.grad, pc.grad) < 4e-2, (n, _rel(pg.grad, pc.grad))


def test_user_step_dropout_changes_with_step_counter(dev):
    torch.manual_seed(1)
    ue = FedRecModel(FedRecConfig()).user_encoder.to(dev)
    D, B, C, H = 400, 4, 5, 50
    uniq, inv, perm, ptr = ops.dedup(torch.randint(0, 100, (B * (C + H),), dtype=torch.int32, device=dev), 100)
    v = torch.randn(uniq.numel(), D, device=dev) * 0.05
    U = uniq.numel()
    rng = torch.zeros(1, dtype=torch.int64, device=dev)
    with torch.no_grad():
        l0, _ = OF.user_step(v, inv, perm, ptr, ue, B, C, H, "sigmoid", (0.2, 9, 0), rng, (0.0, 0.0, 0, 0), False)
        l0b, _ = OF.user_step(v, inv, perm, ptr, ue, B, C, H, "sigmoid", (0.2, 9, 0), rng, (0.0, 0.0, 0, 0), False)
        rng.add_(1)
        l1, _ = OF.user_step(v, inv, perm, ptr, ue, B, C, H, "sigmoid", (0.2, 9, 0), rng, (0.0, 0.0, 0, 0), False)
    assert float(l0) == float(l0b) and float(l0) != float(l1)


def test_head_fc_matches_torch(dev):
    torch.manual_seed(2)
    x = torch.randn(1565, 768, device=dev, requires_grad=True)
    w = (torch.randn(400, 768, device=dev) * 0.03).requires_grad_(True)
    b = torch.randn(400, device=dev, requires_grad=True)
    y = OF.HeadFCFn.apply(x, w, b)
    g = torch.randn_like(y)
    y.backward(g)
    xc, wc, bc = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    yc = torch.nn.functional.linear(xc, wc, bc)
    yc.backward(g)
    assert _rel(y, yc) < 5e-3
    assert _rel(x.grad, xc.grad) < 5e-3 and _rel(w.grad, wc.grad) < 5e-3 and _rel(b.grad, bc.grad) < 1e-5


def test_gather_dropout_matches_oracle():
    """X' = v[idx] o Z on the device == the Philox torch oracle, bit for bit (with the graph
    replay counter dev_off added to the offset)."""
    dev = torch.device("cuda")
    v = torch.randn(300, 400, device=dev)
    idx = torch.randint(0, 300, (3200,), device=dev, dtype=torch.int32)
    dev_off = torch.tensor([7], device=dev, dtype=torch.int64)
    x = ops.gather_dropout(v, idx, 0.2, 11, 5, dev_off)
    xr = ops.gather_dropout(v.cpu(), idx.cpu(), 0.2, 11, 5, dev_off.cpu())
    assert torch.equal(x.cpu(), xr)
    keep = (x != 0).float().mean().item()
    assert abs(keep - 0.8) < 0.01
    assert torch.equal(ops.gather_dropout(v, idx, 0.0, 11, 5, None), v[idx.long()])


@pytest.mark.parametrize("mask", [False, True])
def test_user_encoder_module_on_device_matches_cpu(dev, mask):
    """``UserEncoder.forward`` on the device (OF.UserEncoderFn: the step's kernels, no vendor
    GEMM / torch dropout) against the host module: the user vector and every gradient."""
    torch.manual_seed(3)
    cfg = FedRecConfig(mode="grad_avg", mask_padding=mask)
    ue_c = FedRecModel(cfg).user_encoder
    ue_g = copy.deepcopy(ue_c).to(dev)
    ue_c.eval()
    ue_g.eval()
    B, H, D = 6, 50, 400
    x = torch.randn(B, H, D)  # unit scale: peaky attention, so the pool gradients do not cancel
    his_ids = _his_ids(B, H, dev) if mask else None
    xg = x.to(dev).requires_grad_(True)
    xc = x.clone().requires_grad_(True)
    ug = ue_g(xg, his_ids)
    uc = ue_c(xc, None if his_ids is None else his_ids.cpu())
    g = torch.randn(B, D)
    ug.backward(g.to(dev))
    uc.backward(g)
    assert _rel(ug, uc) < 1e-2, _rel(ug, uc)
    if mask:
        assert float(ug[-1].abs().max()) == 0.0  # every slot padded: the pooled user vector is 0
    assert _rel(xg.grad, xc.grad) < 3e-2
    top = max(float(p.grad.norm()) for p in ue_c.parameters())
    for (n, pg), (_, pc) in zip(ue_g.named_parameters(), ue_c.named_parameters()):
        if float(pc.grad.norm()) < 1e-6 * top:  # a near-cancellation (e.g. the key bias): rounding noise
            assert float(pg.grad.norm()) < 1e-4 * top, n
            continue
        assert _rel(pg.grad, pc.grad) < 4e-2, (n, _rel(pg.grad, pc.grad))
