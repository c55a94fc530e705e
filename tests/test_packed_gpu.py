"""Packed title rows (frozen backbone forward): row plan, row-split QKV GEMM, packed attention,
embedding / LayerNorm row indirection, and the whole backbone against the unpacked path.
Each kernel is compared with a plain PyTorch fp32 reference of the same op."""

import pytest
import torch

from fedrec_with_pytorchdistributed_amd.ops import native
from fedrec_with_pytorchdistributed_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _mask(n, T, g, prefix=True):
    lens = torch.randint(1, T + 1, (n,), generator=g)
    if prefix:
        m = (torch.arange(T)[None, :] < lens[:, None]).to(torch.int32)
    else:  # arbitrary (non-prefix) masks: the plan must not assume left-aligned tokens
        m = (torch.rand(n, T, generator=g) < 0.4).to(torch.int32)
    m[0] = 0  # the <unk> row: every key masked -> uniform attention over all T keys
    return m


@pytest.mark.parametrize("n,T,prefix", [(1577, 50, True), (3, 50, False), (2100, 17, False), (5, 1, True)])
def test_title_plan_matches_oracle(dev, n, T, prefix):
    g = torch.Generator().manual_seed(n * 7 + T)
    m = _mask(n, T, g, prefix)
    got = native.lib().title_plan(m.to(dev))
    want = ref.title_plan(m)
    for a, b, name in zip(got, want, ("rowmap", "src", "kv_start", "kv_len", "qstart", "n_kv")):
        assert torch.equal(a.cpu(), b), name


@pytest.mark.parametrize("n,T,prefix", [(700, 50, True), (40, 50, False), (33, 64, True), (9, 17, False)])
def test_title_attention_packed(dev, n, T, prefix):
    H, D = 12, 768
    g = torch.Generator().manual_seed(n + T)
    m = _mask(n, T, g, prefix)
    qkv = torch.randn(n * T, 3 * D, generator=g).to(torch.bfloat16)
    want = ref.title_attention(qkv.float(), m, H)  # title-major rows
    lib = native.lib()
    rowmap, src, kv_start, kv_len, qstart, n_kv = lib.title_plan(m.to(dev))
    srcl = src.long().cpu()
    packed = qkv[srcl].clone()
    R = int(n_kv.item())
    packed[R:, D:] = float("nan")  # K/V of query-only rows must never be read
    out = lib.title_attention_packed(packed.to(dev), rowmap, kv_start, kv_len, qstart, H)
    got = torch.empty_like(out.cpu())
    got[srcl] = out.cpu()
    assert torch.isfinite(got.float()).all()
    assert rel_err(got, want) < 2e-2


@pytest.mark.parametrize("M,R", [(78850, 25000), (5000, 4097), (4096, 0), (9000, 9000)])
def test_linear_split(dev, M, R):
    K, N = 768, 2304
    g = torch.Generator().manual_seed(M + R)
    x = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
    b = torch.randn(N, generator=g).to(dev)
    lib = native.lib()
    y = lib.linear_split(x, w, b, torch.tensor([R], dtype=torch.int32, device=dev), 768)
    full = lib.linear(x, w, b, 0, None)
    assert torch.equal(y[:, :768], full[:, :768])  # Q columns: every row, same kernel, same order
    assert torch.equal(y[:R], full[:R])  # all columns of the rows read as keys/values
    sl = slice(0, min(M, 2048))
    assert rel_err(full[sl], x[sl].float() @ w.float().t() + b) < 1e-2


def test_embed_rows_and_scatter_ln(dev):
    n, T, D = 300, 50, 768
    g = torch.Generator().manual_seed(3)
    m = _mask(n, T, g)
    tok = torch.randint(0, 30522, (n, T), generator=g, dtype=torch.int32)
    word = (torch.randn(30522, D, generator=g) * 0.02).to(dev, torch.bfloat16)
    pos = (torch.randn(512, D, generator=g) * 0.02).to(dev, torch.bfloat16)
    w, b = torch.randn(D, generator=g).to(dev), torch.randn(D, generator=g).to(dev)
    lib = native.lib()
    _, src, _, _, _, _ = lib.title_plan(m.to(dev))
    e = lib.embed_ln_rows(tok.to(dev), src, word, pos, w, b, 1e-12)
    e_ref = lib.embed_ln(tok.to(dev), word, pos, w, b, 1e-12)
    assert torch.equal(e, e_ref[src.long()])
    x = torch.randn(n * T, D, generator=g).to(dev, torch.bfloat16)
    r = torch.randn(n * T, D, generator=g).to(dev, torch.bfloat16)
    y = lib.layer_norm_scatter(x, w, b, 1e-12, r, src)
    y_ref = lib.layer_norm(x, w, b, 1e-12, r)
    assert torch.equal(y[src.long()], y_ref)


def test_backbone_packed_matches_unpacked(dev):
    """Whole 6-layer DistilBERT forward: packed rows vs the plain layout, on MIND-like titles
    (the synthetic generator's [CLS] w.. [SEP] 0.. rows, plus the all-zero <unk> row)."""
    from fedrec_with_pytorchdistributed_amd.config import FedRecConfig
    from fedrec_with_pytorchdistributed_amd.data.synthetic import make_client_shards
    from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel

    torch.manual_seed(0)
    model = FedRecModel(FedRecConfig()).to(dev)
    te = model.text_encoder
    shard = make_client_shards("tiny", 1)[0]
    text = torch.as_tensor(shard.news_index[:800], dtype=torch.int32).to(dev)
    from fedrec_with_pytorchdistributed_amd.models import backbone as bb

    try:
        bb.TITLE_PACK = False
        h0 = te.hidden(text)
        bb.TITLE_PACK = True
        h1 = te.hidden(text)
    finally:
        bb.TITLE_PACK = True
    assert torch.isfinite(h1.float()).all()
    assert rel_err(h1, h0) < 1e-2
    v0, v1 = te.head(h0), te.head(h1)
    assert rel_err(v1, v0) < 1e-2
