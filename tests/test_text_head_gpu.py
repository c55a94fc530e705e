"""The fused text head (csrc/text_head.hip, ops.functional.TextHeadFn) against the plain-PyTorch
fp32 oracle of the reference head (encoder.py:27-29, attention.py:14-26): titles read from a
hidden-state table by index (duplicates, padded slots of id 0, an all-padding title), forward
(pooled) and every gradient (att_fc1 weight / bias, att_fc2 weight / bias), with and without the
padding-token mask, T = 50 and shorter titles, and a row count that is not a tile multiple."""
import math

import pytest
import torch

from fedrec_with_pytorchdistributed_amd.ops import functional as OF
from fedrec_with_pytorchdistributed_amd.ops import native

pytestmark = pytest.mark.gpu


def _oracle(table, ids, T, w1, b1, w2, b2, tokens):
    """fp32 reference head over table rows (bf16 inputs and bf16 W1 as the kernel consumes them)."""
    D = table.shape[1]
    x = table.view(-1, T, D)[ids.long()].float()  # [U, T, D]
    e = torch.tanh(x @ w1.to(torch.bfloat16).float().t() + b1)
    a = (e @ w2.reshape(-1, 1)).squeeze(-1) + b2
    if tokens is not None:
        keep = tokens[ids.long(), 1, :] != 0
        m = a.masked_fill(~keep, float("-inf")).amax(1, keepdim=True)
        m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
        p = torch.exp(a - m) * keep
    else:
        m = a.amax(1, keepdim=True)
        p = torch.exp(a - m)
    alpha = p / (p.sum(1, keepdim=True) + 1e-8 * torch.exp(-m))
    return torch.einsum("ut,utd->ud", alpha, x)


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / (b.norm() + 1e-20))


@pytest.mark.parametrize("U,T,masked,D", [(257, 50, False, 768), (257, 50, True, 768), (40, 17, False, 768),
                                          (3, 50, False, 768), (1664, 50, False, 768), (40, 64, False, 768),
                                          (30, 100, True, 768), (20, 128, False, 768),
                                          (257, 50, True, 256), (1000, 50, False, 512), (30, 96, False, 1024)])
def test_fused_text_head_matches_fp32_oracle(dev, U, T, masked, D):
    """(D = 256 / 512: Q = 128 / 256, head_score2's 128-row form and the round-4 weight gradient;
    D = 1024 at T = 96: the widest head_pool2 form)"""
    g = torch.Generator(device="cpu").manual_seed(U * 100 + T)
    N, Q = 300, D // 2 if D < 768 else 384
    table = torch.randn(N * T, D, generator=g).to(dev, torch.bfloat16)
    ids = torch.randint(0, N, (U,), generator=g, dtype=torch.int32)
    ids[: min(U, 5)] = 0  # padded slots (the step graphs pad the unique list with news 0)
    ids = ids.to(dev)
    tokens = None
    if masked:
        lens = torch.randint(0, T + 1, (N,), generator=g)
        lens[0] = 0  # the <unk> / pad title: every token masked
        mask = (torch.arange(T).unsqueeze(0) < lens.unsqueeze(1)).to(torch.int32)
        tokens = torch.stack([mask * 7, mask], 1).contiguous().to(dev)
    w1 = (torch.randn(Q, D, generator=g) / math.sqrt(D)).to(dev).requires_grad_(True)
    b1 = (torch.randn(Q, generator=g) * 0.1).to(dev).requires_grad_(True)
    w2 = (torch.randn(1, Q, generator=g) / math.sqrt(Q) * 3).to(dev).requires_grad_(True)
    b2 = torch.randn(1, generator=g).to(dev).requires_grad_(True)
    assert OF.fused_head_supported(D, Q, T)
    pooled, _ = OF.TextHeadFn.apply(w1, b1, w2, b2, table, ids, T, tokens)
    gout = torch.randn(U, D, generator=g).to(dev)
    gw = torch.autograd.grad(pooled, (w1, b1, w2, b2), gout)
    params = [t.detach().clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
    ref = _oracle(table, ids, T, *params, tokens)
    rw = torch.autograd.grad(ref, params, gout)
    torch.cuda.synchronize()
    assert pooled.shape == (U, D) and pooled.dtype == torch.float32
    assert _rel(pooled, ref) < 2e-3, _rel(pooled, ref)
    if masked:  # the all-padding title pools to exactly zero
        z = (ids == 0).nonzero().reshape(-1)
        assert float(pooled.detach()[z].abs().max()) == 0.0
    for name, a, b in zip(("dW1", "db1", "dw2"), gw[:3], rw[:3]):
        assert a.shape == b.shape, name
        assert torch.isfinite(a).all(), name
        assert _rel(a, b) < 3e-2, (name, _rel(a, b))
    # db2 = (1 - sum alpha) sum alpha dalpha per title: ~1e-8 of the other gradients, both sides
    # are fp32 cancellation noise -- bound it against the gradient scale instead
    assert float((gw[3] - rw[3]).abs().max()) < 1e-3 * float(rw[2].norm()), (gw[3], rw[3])


def test_fused_head_forward_only_skips_e(dev):
    """Under no_grad nothing is stored for a backward (validation / epoch news tables)."""
    T, D, Q, U = 50, 768, 384, 100
    table = torch.randn(U * T, D, device=dev).to(torch.bfloat16)
    lib = native.lib()
    w1 = torch.randn(Q, D, device=dev).to(torch.bfloat16)
    b1, w2, b2 = torch.zeros(Q, device=dev), torch.randn(Q, device=dev), torch.zeros(1, device=dev)
    e, a = lib.head_score(table, None, T, w1, b1, w2, b2, False)
    e2, a2 = lib.head_score(table, None, T, w1, b1, w2, b2, True)
    assert e.numel() == 0 and e2.shape == (U * T, Q)
    assert torch.equal(a, a2)
    a2 = a2.reshape(-1, U * T).sum(0)  # [slices, U*T] partial scores of a Q-sliced tiling
    # the score is the row-dot of the fp32 tanh values: agrees with the stored bf16 e to its rounding
    assert _rel(a2 - b2, e2.float() @ w2) < 1e-2


def test_engine_head_uses_fused_kernels_over_cache(dev):
    """The engine's per-step head reads the cache by index (no hidden-row gather) and gives the
    same news vectors and head gradients as the round-2 path (gather + GEMM + pool)."""
    import copy
    import os

    from fedrec_with_pytorchdistributed_amd.config import BackboneConfig, FedRecConfig
    from fedrec_with_pytorchdistributed_amd.data.synthetic import make_client_shards
    from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
    from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine

    cfg = FedRecConfig(mode="grad_avg", batch_size=8, user_dropout=0.0)
    cfg.backbone = BackboneConfig(name="distilbert-2l", n_layers=2)
    torch.manual_seed(0)
    m = FedRecModel(cfg).to(dev)
    m.build_flat()
    shard = make_client_shards("tiny", 1)[0]
    eng = LocalEngine(cfg, m, shard, dev)
    assert eng.fused_head
    ids = torch.tensor([0, 3, 3, 7, 1, 0], dtype=torch.int32, device=dev)
    v = eng.news_vectors(ids, grad=True)
    gv = torch.randn_like(v)
    te = m.text_encoder
    params = [te.additive_attention.att_fc1.weight, te.additive_attention.att_fc1.bias,
              te.additive_attention.att_fc2.weight, te.additive_attention.att_fc2.bias, te.fc.weight, te.fc.bias]
    g1 = torch.autograd.grad(v, params, gv)
    OF.FUSED_HEAD = False
    try:
        te2 = copy.deepcopy(te)
        te2.__dict__.pop("_fused_ok", None)
        hid = eng.hcache.rows(ids)
        v2 = te2.head(hid, None)
        params2 = [te2.additive_attention.att_fc1.weight, te2.additive_attention.att_fc1.bias,
                   te2.additive_attention.att_fc2.weight, te2.additive_attention.att_fc2.bias, te2.fc.weight,
                   te2.fc.bias]
        g2 = torch.autograd.grad(v2, params2, gv)
    finally:
        OF.FUSED_HEAD = True
    assert _rel(v, v2) < 5e-3
    for i, (a, b) in enumerate(zip(g1, g2)):
        if i == 3:  # att_fc2.bias: cancellation noise on both paths (see the oracle test)
            assert float((a - b).abs().max()) < 1e-3 * float(g2[2].norm())
        else:
            assert _rel(a, b) < 3e-2, (i, _rel(a, b))


def test_fused_head_skips_padded_titles(dev):
    """A step graph pads its unique-title list; with the device count ``nreal`` the head kernels
    skip the padded titles: their pooled rows are exactly 0 and they add nothing to the weight
    gradients (which equal the oracle over the real titles alone, whatever gradient arrives for
    the padded rows)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    N, D, Q, T, U, R = 400, 768, 384, 50, 300, 213  # R real titles, U - R padding (id 0)
    table = torch.randn(N * T, D, generator=g).to(dev, torch.bfloat16)
    ids = torch.randint(1, N, (U,), generator=g, dtype=torch.int32)
    ids[R:] = 0
    ids = ids.to(dev)
    nreal = torch.tensor([R], dtype=torch.int32, device=dev)
    w1 = (torch.randn(Q, D, generator=g) / math.sqrt(D)).to(dev).requires_grad_(True)
    b1 = (torch.randn(Q, generator=g) * 0.1).to(dev).requires_grad_(True)
    w2 = (torch.randn(1, Q, generator=g) / math.sqrt(Q) * 3).to(dev).requires_grad_(True)
    b2 = torch.randn(1, generator=g).to(dev).requires_grad_(True)
    pooled, _ = OF.TextHeadFn.apply(w1, b1, w2, b2, table, ids, T, None, nreal)
    gout = torch.randn(U, D, generator=g).to(dev)  # padded rows get a nonzero gradient too
    gw = torch.autograd.grad(pooled, (w1, b1, w2, b2), gout)
    params = [t.detach().clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
    ref = _oracle(table, ids[:R], T, *params, None)
    rw = torch.autograd.grad(ref, params, gout[:R])
    torch.cuda.synchronize()
    assert float(pooled.detach()[R:].abs().max()) == 0.0
    assert _rel(pooled[:R], ref) < 2e-3
    for name, a, b in zip(("dW1", "db1", "dw2"), gw[:3], rw[:3]):
        assert _rel(a, b) < 3e-2, (name, _rel(a, b))


def test_fc_on_bf16_operands_matches_fp32_operands(dev):
    """The fc GEMMs on the pool's bf16 rows and the cast fc weight give the same products as on
    the fp32 pooled rows / fp32 weight (the GEMMs round fp32 operands to bf16 themselves): every
    gradient bitwise; the forward up to fp32 summation order (the bf16 x bf16 launch runs on the
    LDS-DMA ring, which splits K = 768 in one piece where the fp32-operand kernel takes two)."""
    g = torch.Generator(device="cpu").manual_seed(5)
    U, D, N = 333, 768, 400
    x = torch.randn(U, D, generator=g).to(dev).requires_grad_(True)
    w = (torch.randn(N, D, generator=g) / 30).to(dev).requires_grad_(True)
    b = torch.randn(N, generator=g).to(dev).requires_grad_(True)
    dy = torch.randn(U, N, generator=g).to(dev)
    y0 = OF.HeadFCFn.apply(x, w, b)
    gx0, gw0, gb0 = torch.autograd.grad(y0, (x, w, b), dy)
    y1 = OF.HeadFCFn.apply(x, w, b, x.detach().to(torch.bfloat16), w.detach().to(torch.bfloat16))
    gx1, gw1, gb1 = torch.autograd.grad(y1, (x, w, b), dy)
    assert _rel(y0, y1) < 1e-6, _rel(y0, y1)
    assert torch.equal(gx0, gx1) and torch.equal(gw0, gw1) and torch.equal(gb0, gb1)
    # the pool's bf16 output is the fp32 pooled rows rounded
    lib = native.lib()
    T = 50
    table = torch.randn(40 * T, D, generator=g).to(dev, torch.bfloat16)
    ids = torch.randint(0, 40, (17,), generator=g).to(dev, torch.int32)
    a = torch.randn(17 * T, generator=g).to(dev)
    pooled, _, pb = lib.head_pool(table, ids, T, a, None, None, True)
    assert torch.equal(pb, pooled.to(torch.bfloat16))


@pytest.mark.parametrize("U,T", [(1664, 50), (257, 50), (40, 17)])
def test_score_row_tiles_agree_bitwise(dev, U, T):
    """head_score2's 160- and 192-row tiles (the launcher picks by its rounds rule) give the
    same scores and e bit for bit: a row's k order does not depend on the tile."""
    g = torch.Generator(device="cpu").manual_seed(U)
    N, D, Q = 300, 768, 384
    table = torch.randn(N * T, D, generator=g).to(dev, torch.bfloat16)
    ids = torch.randint(0, N, (U,), generator=g, dtype=torch.int32).to(dev)
    w1 = (torch.randn(Q, D, generator=g) / math.sqrt(D)).to(dev, torch.bfloat16)
    b1, w2 = (torch.randn(Q, generator=g) * 0.1).to(dev), (torch.randn(Q, generator=g) / 20).to(dev)
    b2 = torch.randn(1, generator=g).to(dev)
    lib = native.lib()
    outs = []
    try:
        for rows in (192, 160):
            for ilv in (0, 1):  # (the next stage's loads interleaved with the MFMAs: no arithmetic change)
                lib.head_score_set_rows(rows)
                lib.head_score_set_ilv(ilv)
                outs.append(lib.head_score(table, ids, T, w1, b1, w2, b2, True))
    finally:
        lib.head_score_set_rows(0)
        lib.head_score_set_ilv(1)
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1])


@pytest.mark.parametrize("U,T,padded", [(1577, 50, True), (257, 50, False), (40, 17, False), (30, 100, True)])
def test_head_g_path_matches_round4_path(dev, U, T, padded):
    """The G path (pool backward writes g = da (1 - e^2) and the per-title column sums, the weight
    gradient is a plain TN GEMM over g: head_pool_bwd_g + head_wgrad_g) against the round-4 path
    (the rewrite inside head_wgrad's LDS pipeline).  Both consume the same bf16 g values, so the
    gradients agree to fp32 summation order; padded titles (nreal) are skipped on both."""
    g = torch.Generator(device="cpu").manual_seed(U + T)
    N, D, Q = 2000, 768, 384
    table = torch.randn(N * T, D, generator=g).to(dev, torch.bfloat16)
    ids = torch.randint(1, N, (U,), generator=g, dtype=torch.int32)
    R = U - 37 if padded else U
    ids[R:] = 0
    ids = ids.to(dev)
    nreal = torch.tensor([R], dtype=torch.int32, device=dev) if padded else None
    w1 = (torch.randn(Q, D, generator=g) / math.sqrt(D)).to(dev).requires_grad_(True)
    b1 = (torch.randn(Q, generator=g) * 0.1).to(dev).requires_grad_(True)
    w2 = (torch.randn(1, Q, generator=g) / math.sqrt(Q) * 3).to(dev).requires_grad_(True)
    b2 = torch.randn(1, generator=g).to(dev).requires_grad_(True)
    gout = torch.randn(U, D, generator=g).to(dev)
    lib = native.lib()
    assert lib.head_g_supported(D, Q, T)
    w1b = w1.detach().to(torch.bfloat16)
    w2f = w2.detach().reshape(-1).contiguous()
    e, a = lib.head_score(table, ids, T, w1b, b1.detach(), w2f, b2.detach().reshape(-1), True, nreal)
    _, alpha, _ = lib.head_pool(table, ids, T, a, None, nreal, False)
    out = {}
    eg = e.clone()  # (the G path rewrites e into g in place)
    da, db2p, cs = lib.head_pool_bwd_g(table, ids, T, alpha, gout, eg, nreal)
    out["1"] = lib.head_wgrad_g(table, ids, T, eg, cs, w2f, db2p, nreal)
    da0, db2p0 = lib.head_pool_bwd(table, ids, T, alpha, gout, nreal)
    out["0"] = lib.head_wgrad(table, ids, T, e, da0, w2f, db2p0, nreal)
    torch.cuda.synchronize()
    for name, a_, b_ in zip(("dW1", "db1", "dw2"), out["1"][:3], out["0"][:3]):
        assert torch.isfinite(a_).all(), name
        assert _rel(a_, b_) < 1e-4, (name, _rel(a_, b_))
    assert float((out["1"][3] - out["0"][3]).abs().max()) <= 1e-6 * float(out["0"][2].norm()) + 1e-7


@pytest.mark.parametrize("U,padded", [(1577, True), (300, False), (7, False)])
def test_head_wgrad_g_matches_fp32(dev, U, padded):
    """head_wgrad_g (a plain TN GEMM over g with the cache rows by title index, whole-title
    splits, padded titles skipped) against an fp32 matmul of the same bf16 operands; the column
    partials cs are summed over the real titles only."""
    g = torch.Generator(device="cpu").manual_seed(U)
    N, D, Q, T = 2000, 768, 384, 50
    lib = native.lib()
    table = torch.randn(N * T, D, generator=g).to(dev, torch.bfloat16)
    ids = torch.randint(1, N, (U,), generator=g, dtype=torch.int32).to(dev)
    R = U - 50 if padded else U
    nreal = torch.tensor([R], dtype=torch.int32, device=dev) if padded else None
    G = (torch.randn(U * T, Q, generator=g) * 0.1).to(dev, torch.bfloat16)
    cs = torch.randn(2, U, Q, generator=g).to(dev)
    w2 = torch.randn(Q, generator=g).to(dev)
    db2p = torch.randn(U, generator=g).to(dev)
    dW1, db1, dw2, db2 = lib.head_wgrad_g(table, ids, T, G, cs, w2, db2p, nreal)
    torch.cuda.synchronize()
    x = table.view(N, T, D)[ids[:R].long()].reshape(-1, D).float()
    ref = G[: R * T].float().t() @ x * w2.view(-1, 1)
    assert _rel(dW1, ref) < 1e-5, _rel(dW1, ref)
    assert _rel(dw2, cs[0, :R].sum(0)) < 1e-5
    assert _rel(db1, cs[1, :R].sum(0) * w2) < 1e-5
    assert abs(float(db2) - float(db2p.sum())) < 1e-3


@pytest.mark.parametrize("U,T,padded", [(1577, 50, True), (257, 50, False), (40, 17, False), (30, 100, True)])
def test_head_pool_bwd_g_matches_pool_bwd_and_oracle(dev, U, T, padded):
    """head_pool_bwd_g (pool backward + the g rewrite of the title's e rows + its column partials
    in one launch, e loaded after the X rows are consumed): da / db2p bitwise head_pool_bwd's
    (same arithmetic, same order); g = da (1 - e^2) rounded to bf16 and the per-title column
    partials cs[0] = sum_t da_t e_t, cs[1] = sum_t g_t against an fp32 torch oracle."""
    g = torch.Generator(device="cpu").manual_seed(3 * U + T)
    N, D, Q = 2000, 768, 384
    lib = native.lib()
    table = torch.randn(N * T, D, generator=g).to(dev, torch.bfloat16)
    ids = torch.randint(1, N, (U,), generator=g, dtype=torch.int32)
    R = U - 11 if padded else U
    ids[R:] = 0
    ids = ids.to(dev)
    nreal = torch.tensor([R], dtype=torch.int32, device=dev) if padded else None
    alpha = torch.softmax(torch.randn(U, T, generator=g), 1).to(dev)
    gp = torch.randn(U, D, generator=g).to(dev)
    e0 = torch.tanh(torch.randn(U * T, Q, generator=g)).to(dev, torch.bfloat16)
    e1 = e0.clone()
    da1, db1, cs1 = lib.head_pool_bwd_g(table, ids, T, alpha, gp, e1, nreal)
    da2, db2 = lib.head_pool_bwd(table, ids, T, alpha, gp, nreal)
    torch.cuda.synchronize()
    assert torch.equal(da1, da2) and torch.equal(db1, db2)
    n = R * T
    ef = e0[:n].float()
    dav = da2.reshape(-1)[:n].view(-1, 1)
    gref = (dav * (1.0 - ef * ef)).to(torch.bfloat16)
    # one bf16 ulp: the kernel's fp32 expression may round once differently before the cast
    assert float(((e1[:n].float() - gref.float()).abs() - gref.float().abs() * 2 ** -7).max()) <= 1e-30
    cs0 = (dav * ef).view(R, T, Q).sum(1)
    cs1r = gref.float().view(R, T, Q).sum(1)
    assert _rel(cs1[0, :R], cs0) < 1e-5, _rel(cs1[0, :R], cs0)
    assert _rel(cs1[1, :R], cs1r) < 1e-4, _rel(cs1[1, :R], cs1r)
