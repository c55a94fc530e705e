"""Numerics of every HIP kernel against the plain-PyTorch fp32 oracle (ops/reference.py).

bf16 kernels are compared with tolerances scaled to bf16 rounding; fp32 kernels tightly.
"""
import math

import pytest
import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.ops import native
from fedrec_with_pytorchdistributed_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("M,N,K,act,res", [(1000, 2304, 768, "none", False), (777, 768, 3072, "none", True),
                                           (256, 3072, 768, "gelu", False), (130, 384, 768, "tanh", False),
                                           (5, 128, 64, "none", True)])
def test_gemm_bf16(dev, M, N, K, act, res):
    g = torch.Generator(device="cpu").manual_seed(M + N)
    x = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(dev, torch.bfloat16)
    b = torch.randn(N, generator=g).to(dev)
    r = torch.randn(M, N, generator=g).to(dev, torch.bfloat16) if res else None
    y = native.lib().linear(x, w, b, {"none": 0, "gelu": 1, "tanh": 2}[act], r)
    y_ref = ref.linear(x.float(), w.float(), b, act, r.float() if res else None)
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert rel_err(y, y_ref) < 1e-2


def test_gemm_asymmetric_exact(dev):
    # A = I-like, asymmetric B: catches row/col swaps in the C write (guide §3)
    M = N = 128
    K = 128
    x = torch.eye(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.arange(N * K, device=dev, dtype=torch.float32).remainder(97).reshape(N, K).to(torch.bfloat16)
    y = native.lib().linear(x, w, None, 0, None)
    assert torch.equal(y.float(), w.float().t())


def test_layer_norm(dev):
    x = torch.randn(333, 768, device=dev).to(torch.bfloat16) * 3 + 1
    w = torch.randn(768, device=dev)
    b = torch.randn(768, device=dev)
    y = native.lib().layer_norm(x, w, b, 1e-12)
    assert rel_err(y, ref.layer_norm(x.float(), w, b, 1e-12)) < 1e-2


@pytest.mark.parametrize("wide", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("rows,D", [(1, 768), (333, 768), (77, 512), (5000, 768)])
def test_layer_norm_forms(dev, wide, rows, D):
    x = torch.randn(rows, D, device=dev).to(torch.bfloat16) * 3 + 1
    w, b = torch.randn(D, device=dev), torch.randn(D, device=dev)
    lib = native.lib()
    lib.ln_set_wide(wide)
    try:
        y = lib.layer_norm(x, w, b, 1e-12)
        word = (torch.randn(1000, D, device=dev) * 0.5).to(torch.bfloat16)
        pos = (torch.randn(64, D, device=dev) * 0.5).to(torch.bfloat16)
        tok = torch.randint(0, 1000, (rows,), device=dev, dtype=torch.int32)
        e = lib.embed_ln(tok.view(rows, 1), word, pos, w, b, 1e-12)
    finally:
        lib.ln_set_wide(4)
    assert rel_err(y, ref.layer_norm(x.float(), w, b, 1e-12)) < 1e-2
    r = torch.randn(rows, D, device=dev).to(torch.bfloat16)
    lib.ln_set_wide(wide)
    try:
        yr = lib.layer_norm(x, w, b, 1e-12, r)
    finally:
        lib.ln_set_wide(4)
    assert rel_err(yr, ref.layer_norm(x.float() + r.float(), w, b, 1e-12)) < 1e-2
    e_ref = ref.embed_ln(tok.view(rows, 1).long(), word.float(), pos.float(), w, b, 1e-12)
    assert rel_err(e, e_ref) < 1e-2


def test_embed_ln(dev):
    n, T, D = 37, 50, 768
    word = (torch.randn(30522, D, device=dev) * 0.02).to(torch.bfloat16)
    pos = (torch.randn(512, D, device=dev) * 0.02).to(torch.bfloat16)
    tok = torch.randint(0, 30522, (n, T), device=dev, dtype=torch.int32)
    w, b = torch.randn(D, device=dev), torch.randn(D, device=dev)
    y = native.lib().embed_ln(tok, word, pos, w, b, 1e-12)
    y_ref = ref.embed_ln(tok.long(), word.float(), pos.float(), w, b, 1e-12)
    assert rel_err(y, y_ref) < 1e-2


@pytest.mark.parametrize("T", [50, 64, 17, 1, 65, 130, 512])
def test_title_attention(dev, T):
    """T > 64 runs title_attn_long.hip (online softmax over 64-key LDS chunks, up to 512)."""
    n, H, D = 9, 12, 768
    qkv = torch.randn(n * T, 3 * D, device=dev).to(torch.bfloat16)
    mask = (torch.rand(n, T, device=dev) < 0.7).to(torch.int32)
    mask[:, 0] = 1
    mask[0] = 0  # the <unk> row: all keys masked -> uniform (HF finfo.min semantics)
    out = native.lib().title_attention(qkv, mask, H)
    out_ref = ref.title_attention(qkv.float(), mask, H)
    assert torch.isfinite(out.float()).all()
    assert rel_err(out, out_ref) < 2e-2


@pytest.mark.parametrize("waves", [-2, -1, 0, 1, 2, 4])
@pytest.mark.parametrize("n,T", [(700, 50), (3, 33)])
def test_title_attention_launch_variants(dev, waves, n, T):
    """Every launch form (persistent prefetching with 1 or 2 waves/SIMD; 1/2/4 waves per
    block) on enough titles that each persistent wave walks several (title, head) pairs."""
    H, D = 12, 768
    g = torch.Generator().manual_seed(n + T)
    qkv = torch.randn(n * T, 3 * D, generator=g).to(dev, torch.bfloat16)
    lens = torch.randint(1, T + 1, (n,), generator=g)
    mask = (torch.arange(T)[None, :] < lens[:, None]).to(torch.int32).to(dev)
    mask[0] = 0
    lib = native.lib()
    lib.title_attn_set_waves(waves)
    try:
        out = lib.title_attention(qkv, mask, H)
        assert torch.equal(lib.title_attention(qkv, mask, H), out)
    finally:
        lib.title_attn_set_waves(-2)
    assert torch.isfinite(out.float()).all()
    assert rel_err(out, ref.title_attention(qkv.float(), mask, H)) < 2e-2


@pytest.mark.parametrize("dtype,D,Q", [(torch.bfloat16, 768, 384), (torch.float32, 400, 200), (torch.bfloat16, 64, 32),
                                       (torch.bfloat16, 512, 256)])
def test_additive_pool(dev, dtype, D, Q):
    n, T = 23, 50
    x = torch.randn(n, T, D, device=dev).to(dtype)
    e = torch.tanh(torch.randn(n, T, Q, device=dev)).to(dtype)
    w2 = torch.randn(Q, device=dev) * 0.1
    b2 = torch.randn(1, device=dev)
    out, alpha = ops.additive_pool_fwd(x, e, w2, b2)
    o_ref, a_ref = ref.additive_pool_fwd(x.float(), e.float(), w2, b2)
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    assert rel_err(out, o_ref) < tol and rel_err(alpha, a_ref) < tol
    g = torch.randn(n, D, device=dev)
    dx, dpre, dw2, db2 = ops.additive_pool_bwd(x, e, alpha, w2, g, True)
    rdx, rde, rdw2, rdb2 = ref.additive_pool_bwd(x.float(), e.float(), a_ref, w2, g)
    rdpre = rde * (1 - e.float() ** 2)
    assert rel_err(dx, rdx) < tol
    assert rel_err(dpre, rdpre) < 2 * tol
    assert rel_err(dw2, rdw2) < 2 * tol
    assert abs(float(db2) - float(rdb2)) < 1e-3 * (abs(float(rdb2)) + 1)
    # frozen-backbone form (no dx): the vectorised text-head kernel for bf16
    _, dpre_n, dw2_n, db2_n, dsum = ops.additive_pool_bwd(x, e, alpha, w2, g, False, want_colsum=True)
    assert rel_err(dpre_n, rdpre) < 2 * tol
    if dsum is not None:  # fused column sum == sum of the (rounded) dpre it wrote
        assert rel_err(dsum, dpre_n.float().sum((0, 1))) < 1e-4
    assert rel_err(dw2_n, rdw2) < 2 * tol
    assert abs(float(db2_n) - float(rdb2)) < 1e-3 * (abs(float(rdb2)) + 1)


@pytest.mark.parametrize("H", [1, 17, 33, 50, 64, 65, 76, 200])
def test_user_attention(dev, H):
    """H <= 64: the fp32 matrix-core kernels (v_mfma_f32_16x16x4_f32, four waves per head), held
    to 1e-5 against the fp32 oracle forward AND backward; H > 64 runs the long-history kernels
    (online softmax over 64-row LDS chunks): the reference never truncates histories (Q6; its
    shipped shard has H = 76)."""
    B, NH, DK = 7, 20, 20
    qkv = torch.randn(B, H, 3 * NH * DK, device=dev)
    ctx, stats = ops.user_attention_fwd(qkv, NH, DK)
    d = torch.randn_like(ctx)
    dq = ops.user_attention_bwd(qkv, stats, d, NH, DK)
    c_ref, A = ref.user_attention_fwd(qkv, NH, DK)
    assert rel_err(ctx, c_ref) < 1e-5
    dq_ref = ref.user_attention_bwd(qkv, A, d, NH, DK)
    assert rel_err(dq, dq_ref) < (1e-5 if H <= 64 else 1e-4)


@pytest.mark.parametrize("H,masked", [(50, False), (50, True), (17, False), (64, True), (1, False)])
def test_user_qkv_attention_fused_matches_two_launches(dev, H, masked):
    """The Q|K|V projection inside the attention launch equals the small-GEMM launch followed by
    the attention launch bit for bit (same MFMA products, same k order): qkv, ctx, its bf16 copy
    and the softmax stats; and the fp32 attention oracle on that qkv."""
    B, NH, DK, Din = 9, 20, 20, 400
    D3 = 3 * NH * DK
    torch.manual_seed(H)
    xd = torch.randn(B * H, Din, device=dev).to(torch.bfloat16)
    W = (torch.randn(D3, Din, device=dev) * 0.05).to(torch.bfloat16)
    bias = torch.randn(D3, device=dev)
    keep = (torch.rand(B, H, device=dev) > 0.3).to(torch.int32) if masked else None
    cb1 = torch.empty(B, H, NH * DK, device=dev, dtype=torch.bfloat16)
    ctx1, st1, qkv1 = ops.user_qkv_attention_fwd(xd, W, bias, B, NH, DK, keep, cb1)
    qkv2 = torch.empty(B * H, D3, device=dev)
    ops.small_gemm(ops.Gemm(xd, W, qkv2, B * H, D3, Din, Din, Din, D3, bias=bias))
    cb2 = torch.empty_like(cb1)
    ctx2, st2 = ops.user_attention_fwd(qkv2.view(B, H, D3), NH, DK, keep, cb2)
    assert torch.equal(qkv1.view(-1), qkv2.view(-1))
    assert torch.equal(ctx1, ctx2) and torch.equal(cb1, cb2) and torch.equal(st1, st2)
    c_ref, _ = ref.user_attention_fwd(qkv2.view(B, H, D3), NH, DK, keep=keep)
    assert rel_err(ctx1, c_ref) < 1e-5


@pytest.mark.parametrize("H,masked", [(50, False), (50, True), (17, False), (64, True)])
def test_user_attention_bwd_dctx_fused_matches_two_launches(dev, H, masked):
    """The pool's input-gradient GEMM (dctx += dpre W1) inside the attention backward launch equals
    the register-direct GEMM launch followed by the attention backward bit for bit, and leaves
    dctx_direct unchanged."""
    B, NH, DK, Qd = 9, 20, 20, 200
    D = NH * DK
    torch.manual_seed(H + 1)
    qkv = torch.randn(B, H, 3 * D, device=dev)
    keep = (torch.rand(B, H, device=dev) > 0.3).to(torch.int32) if masked else None
    _, stats = ops.user_attention_fwd(qkv, NH, DK, keep)
    dctx = torch.randn(B, H, D, device=dev)
    dpre = torch.randn(B * H, Qd, device=dev).to(torch.bfloat16)
    w1t = (torch.randn(D, Qd, device=dev) * 0.05).to(torch.bfloat16)
    d0 = dctx.clone()
    got = ops.user_attention_bwd_dctx(qkv, stats, dctx, dpre, w1t, NH, DK, keep)
    assert torch.equal(dctx, d0)
    d2 = dctx.clone()
    ops.small_gemm(ops.Gemm(dpre, w1t, d2.view(B * H, D), B * H, D, Qd, Qd, Qd, D, accumulate=True), tile=1004)
    want = ops.user_attention_bwd(qkv, stats, d2, NH, DK, keep, True)
    assert torch.equal(got, want)


@pytest.mark.parametrize("T", [76, 300])
def test_additive_pool_long_fp32(dev, T):
    """User-side pooling over long (untruncated, Q6) histories: the generic kernels."""
    n, D, Q = 5, 400, 200
    x = torch.randn(n, T, D, device=dev)
    e = torch.tanh(torch.randn(n, T, Q, device=dev))
    w2 = torch.randn(Q, device=dev) * 0.1
    b2 = torch.randn(1, device=dev)
    out, alpha = ops.additive_pool_fwd(x, e, w2, b2)
    o_ref, a_ref = ref.additive_pool_fwd(x, e, w2, b2)
    assert rel_err(out, o_ref) < 1e-5 and rel_err(alpha, a_ref) < 1e-5
    g = torch.randn(n, D, device=dev)
    dx, dpre, dw2, db2 = ops.additive_pool_bwd(x, e, alpha, w2, g, True)
    rdx, rde, rdw2, rdb2 = ref.additive_pool_bwd(x, e, a_ref, w2, g)
    assert rel_err(dx, rdx) < 1e-5 and rel_err(dpre, rde * (1 - e ** 2)) < 1e-4 and rel_err(dw2, rdw2) < 1e-4


@pytest.mark.parametrize("variant", [1, 0])  # 1: block per impression (default), 0: wave per impression
@pytest.mark.parametrize("act,C", [("sigmoid", 5), ("identity", 5), ("sigmoid", 16), ("identity", 1)])
def test_score_ce(dev, variant, act, C):
    B, D = 33, 400
    cand = torch.randn(B, C, D, device=dev) * 0.1
    u = torch.randn(B, D, device=dev) * 0.1
    native.lib().score_set_variant(variant)
    try:  # process-global: restored even when the call fails
        loss, s, dc, du = ops.score_ce(cand, u, act)
    finally:
        native.lib().score_set_variant(1)
    l2, s2, dc2, du2 = ref.score_ce_fwd_bwd(cand, u, act)
    assert abs(float(loss) - float(l2)) < 1e-5
    assert rel_err(s, s2) < 1e-6 and rel_err(dc, dc2) < 1e-5 and rel_err(du, du2) < 1e-5


@pytest.mark.parametrize("num_news", [500, 3 << 20])  # 32-bit sort keys / the 64-bit form (ids >= 2^19)
@pytest.mark.parametrize("R", [64 * 55, 37, 1024, 128 * 55, 8192])  # register-bitonic slots E = 4, 1, 1, 8, 8
def test_dedup_and_segment_sum(dev, num_news, R):
    # (64-bit keys at P = 8192 would need a 128 KB two-buffer key image: the LDS form runs those)
    ids = torch.randint(0, num_news, (R,), device=dev, dtype=torch.int32)
    ids[::7] = ids[3]  # repeated ids: the occurrence order inside a segment must be ascending
    uniq, inv, perm, ptr = ops.dedup(ids, num_news)
    u_ref = torch.unique(ids.cpu())
    assert torch.equal(uniq.cpu().long(), u_ref.long())
    assert torch.equal(uniq[inv.long()], ids)
    order = torch.sort(ids.cpu().long() * ids.numel() + torch.arange(ids.numel()), stable=True).indices
    assert torch.equal(perm.cpu().long(), order)
    rows = torch.randn(ids.numel(), 400, device=dev)
    out = ops.segment_sum_rows(rows, inv, uniq.numel(), seg=(perm, ptr))
    o_ref = ref.segment_sum_rows(rows, inv, uniq.numel())
    assert rel_err(out, o_ref) < 1e-6
    # clipping
    out_c = ops.segment_sum_rows(rows, inv, uniq.numel(), clip=2.0, seg=(perm, ptr))
    oc_ref = ref.segment_sum_rows(rows, inv, uniq.numel(), clip=2.0)
    assert rel_err(out_c, oc_ref) < 1e-5


@pytest.mark.parametrize("variant", [2, 1, 0])
@pytest.mark.parametrize("R,D", [(3521, 400), (37, 400), (16, 64), (2000, 512), (300, 36)])
def test_segment_sum_skewed(dev, variant, R, D):
    """Segment sums with a MIND-like skew (a ~30 % pad-row segment, Zipf-popular ids, many
    singletons; R not a multiple of the 16-row chunk): chunked form (1, default) and the
    block-per-row form (0) against an fp64 index_add, bitwise reproducible run to run; the float4
    chunk pass (2, default) is bitwise the scalar one (1)."""
    g = torch.Generator().manual_seed(R + D)
    ids = torch.multinomial(1.0 / torch.arange(1, 600, dtype=torch.float64), R, replacement=True, generator=g)
    ids[torch.rand(R, generator=g) < 0.3] = 0
    ids = ids.to(torch.int32).to(dev)
    uniq, inv, perm, ptr = ops.dedup(ids, 600)
    rows = torch.randn(R, D, generator=g).to(dev)
    lib = native.lib()
    lib.segsum_set_variant(variant)
    try:
        out = ops.segment_sum_rows(rows, inv, uniq.numel(), seg=(perm, ptr))
        assert torch.equal(ops.segment_sum_rows(rows, inv, uniq.numel(), seg=(perm, ptr)), out)
        if variant == 2:
            lib.segsum_set_variant(1)
            assert torch.equal(ops.segment_sum_rows(rows, inv, uniq.numel(), seg=(perm, ptr)), out)
    finally:
        lib.segsum_set_variant(2)
    o_ref = torch.zeros(uniq.numel(), D, dtype=torch.float64).index_add_(0, inv.long().cpu(), rows.double().cpu())
    assert rel_err(out, o_ref) < 1e-6


@pytest.mark.parametrize("R,D", [(3521, 400), (37, 400), (16, 64), (2000, 512)])
def test_segment_sum_ldp_block_form_matches_wave_form(dev, R, D):
    """The LDP chunk pass with the clip + noise spread over a 256-thread block per chunk (default)
    against the one-wave-per-chunk form: same transform, same summation order -- bitwise."""
    g = torch.Generator().manual_seed(7 * R + D)
    ids = torch.multinomial(1.0 / torch.arange(1, 600, dtype=torch.float64), R, replacement=True, generator=g)
    ids[torch.rand(R, generator=g) < 0.3] = 0
    ids = ids.to(torch.int32).to(dev)
    uniq, inv, perm, ptr = ops.dedup(ids, 600)
    rows = (torch.randn(R, D, generator=g) * 3).to(dev)
    lib = native.lib()
    outs = []
    try:
        for form in (2, 3):  # bit 0: the LDP pass on a block per chunk
            lib.segsum_set_ldp_block(form)
            outs.append(ops.segment_sum_rows(rows, inv, uniq.numel(), clip=2.0, noise_std=0.5, seed=11, offset=3,
                                             seg=(perm, ptr)))
        lib.segsum_set_ldp_block(3)  # the block form for the plain (no LDP) pass as well (default)
        plain_blk = ops.segment_sum_rows(rows, inv, uniq.numel(), seg=(perm, ptr))
        lib.segsum_set_ldp_block(1)
        plain = ops.segment_sum_rows(rows, inv, uniq.numel(), seg=(perm, ptr))
    finally:
        lib.segsum_set_ldp_block(3)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[1]).all()
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(plain_blk, plain)


def test_ldp_noise_statistics(dev):
    R, D = 4096, 400
    rows = torch.zeros(R, D, device=dev)
    inv = torch.arange(R, device=dev, dtype=torch.int32)
    perm, ptr = ops.segments_from_inv(inv, R)
    out = ops.segment_sum_rows(rows, inv, R, clip=2.0, noise_std=3.0, seed=5, offset=1, seg=(perm, ptr))
    assert abs(float(out.mean())) < 0.02
    assert abs(float(out.std()) - 3.0) < 0.03
    out2 = ops.segment_sum_rows(rows, inv, R, clip=2.0, noise_std=3.0, seed=5, offset=1, seg=(perm, ptr))
    assert torch.equal(out, out2)  # counter-based: reproducible
    # element-wise independence: neighbouring elements / rows uncorrelated
    z = out / 3.0
    assert abs(float((z[:, :-1] * z[:, 1:]).mean())) < 0.01
    assert abs(float((z[:-1] * z[1:]).mean())) < 0.01
    out3 = ops.segment_sum_rows(rows, inv, R, clip=2.0, noise_std=3.0, seed=5, offset=2, seg=(perm, ptr))
    assert abs(float((out3 * out).mean()) / 9.0) < 0.01  # new step offset -> fresh noise


def test_segment_sum_skewed_pad_row(dev):
    """The pad/<unk> news id collects most history occurrences in a real batch (one segment
    of ~2000 rows next to hundreds of 1-row segments): exact vs the fp32 oracle."""
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(1, 700, (64 * 55,), generator=g, dtype=torch.int32)
    ids[torch.rand(ids.numel(), generator=g) < 0.6] = 0
    ids = ids.to(dev)
    uniq, inv, perm, ptr = ops.dedup(ids, 700)
    rows = torch.randn(ids.numel(), 400, device=dev)
    out = ops.segment_sum_rows(rows, inv, uniq.numel(), seg=(perm, ptr))
    assert rel_err(out, ref.segment_sum_rows(rows, inv, uniq.numel())) < 1e-6
    out_c = ops.segment_sum_rows(rows, inv, uniq.numel(), clip=1.5, seg=(perm, ptr))
    assert rel_err(out_c, ref.segment_sum_rows(rows, inv, uniq.numel(), clip=1.5)) < 1e-5


def test_wgrad_split_k(dev):
    from fedrec_with_pytorchdistributed_amd.ops.functional import bgrad, wgrad
    for M in (78850, 5000, 999):
        dy = torch.randn(M, 384, device=dev).to(torch.bfloat16)
        x = torch.randn(M, 768, device=dev).to(torch.bfloat16)
        assert rel_err(wgrad(dy, x), dy.float().t() @ x.float()) < 1e-5
        assert rel_err(bgrad(dy), dy.float().sum(0)) < 1e-5


def test_adam_flat(dev):
    n = 4096
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    p2, m2, v2 = p.clone().cpu(), m.clone().cpu(), v.clone().cpu()
    for step in (1, 2, 3):
        ops.adam_flat(p, g, m, v, step, 1e-3, 0.9, 0.999, 1e-8, grad_scale=0.5)
        ref.adam_step(p2, g.cpu(), m2, v2, step, 1e-3, 0.9, 0.999, 1e-8, grad_scale=0.5)
    assert rel_err(p, p2) < 1e-6
    # compare with torch.optim.Adam
    tp = torch.nn.Parameter(torch.ones(8))
    opt = torch.optim.Adam([tp], lr=5e-5)
    fp, fm, fv = torch.ones(8, device=dev), torch.zeros(8, device=dev), torch.zeros(8, device=dev)
    for step in (1, 2):
        tp.grad = torch.full((8,), 0.3)
        opt.step()
        ops.adam_flat(fp, torch.full((8,), 0.3, device=dev), fm, fv, step, 5e-5, 0.9, 0.999, 1e-8)
    assert torch.allclose(fp.cpu(), tp.detach(), atol=1e-7)


def test_secagg_cancels_exactly(dev):
    from fedrec_with_pytorchdistributed_amd.parallel import secagg

    W, n = 4, 10_000
    xs = [torch.randn(n, device=dev) for _ in range(W)]
    seeds = secagg.pair_seeds(W, base_seed=123)
    masked = [secagg.mask_local(xs[i], i, W, seeds, round_idx=3) for i in range(W)]
    total = masked[0].clone()
    for t in masked[1:]:
        total += t  # int32 wrap-around == RCCL int32 SUM
    got = secagg.unmask_sum(total)
    q = [secagg.quantize_ref(x) for x in xs]
    exp = sum(q[1:], q[0].clone())
    assert torch.equal(got, secagg.dequantize_ref(exp))


def test_secagg_exact_kernels_match_host(dev):
    """The exact secure sum's device kernels against the host protocol, one client's view with
    no peers (no masks): the exponent histogram equals the host one-hot (+ non-finite count),
    and mask -> unmask is round(x 2^f) 2^-f with the host's f."""
    import numpy as np

    from fedrec_with_pytorchdistributed_amd.ops import native
    from fedrec_with_pytorchdistributed_amd.parallel import secagg

    lib = native.lib()
    sd = torch.zeros(0, dtype=torch.int64, device=dev)
    sg = torch.zeros(0, dtype=torch.int32, device=dev)
    for scale in (0.0, 1e-30, 3e-3, 1.0, 7.5e5):
        x = torch.randn(50_001, device=dev) * scale
        x[17] = 2.0 * scale  # a known maximum
        h = lib.secagg_hist(x, sd, sg, 5).cpu().numpy()
        assert np.array_equal(h, secagg.hist_local(x.cpu()).astype(np.int32)), scale
        for W in (1, 3, 8):
            f, bad = secagg.hist_frac_bits(h, W)
            q = lib.secagg_mask_exact(x, sd, sg, torch.from_numpy(h).to(dev), W, 5)
            exp = torch.round(x.double().cpu() * 2.0 ** f)
            assert torch.equal(q.cpu().double(), exp), (scale, W)
            out = torch.empty_like(x)
            lib.secagg_unmask_exact_(q, torch.from_numpy(h).to(dev), W, out)
            assert torch.equal(out.cpu(), (exp * 2.0 ** -f).float()) and not bad
    x = torch.zeros(1000, device=dev)
    x[3], x[9] = float("nan"), float("inf")
    h = lib.secagg_hist(x, sd, sg, 5)
    assert int(h[1]) == 2 and int(h[0]) == 1
    out = torch.empty_like(x)
    lib.secagg_unmask_exact_(lib.secagg_mask_exact(x, sd, sg, h, 2, 5), h, 2, out)
    assert bool(torch.isnan(out).all())


# -1 auto (variant 12 on no-residual N % 256 shapes), 0 the 128x128 kernel, 6 / 9 the ping-pong
# forms, 12 bias-armed accumulators, 13 = 12 with non-temporal stores
@pytest.mark.parametrize("variant", [-1, 0, 6, 9, 12, 13])
@pytest.mark.parametrize("M,N,K,act,res,bias", [(5000, 768, 768, "none", True, True), (4133, 2304, 768, "gelu", False, True),
                                                (70000, 768, 3072, "none", True, True),
                                                (78850, 2304, 768, "none", False, True),
                                                (20000, 3072, 768, "gelu", False, True), (9000, 768, 3072, "none", False, False),
                                                (300, 256, 64, "tanh", True, True), (78850, 384, 768, "tanh", False, True),
                                                (12345, 512, 768, "tanh", False, False)])
def test_gemm_variants(dev, variant, M, N, K, act, res, bias):
    lib = native.lib()
    g = torch.Generator(device="cpu").manual_seed(M)
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(dev, torch.bfloat16)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5).to(dev, torch.bfloat16)
    b = torch.randn(N, generator=g).to(dev) if bias else None
    r = torch.randn(M, N, generator=g).to(dev, torch.bfloat16) if res else None
    lib.gemm_set_variant(variant)
    try:
        y = lib.linear(x, w, b, {"none": 0, "gelu": 1, "tanh": 2}[act], r)
        # race screen: the pipelined variants must be bitwise deterministic run to run
        for _ in range(3):
            assert torch.equal(lib.linear(x, w, b, {"none": 0, "gelu": 1, "tanh": 2}[act], r), y)
    finally:
        lib.gemm_set_variant(-1)
    # fp32 reference on device (exact erf GELU)
    y_ref = torch.nn.functional.linear(x.float(), w.float(), b)
    if act == "gelu":
        y_ref = torch.nn.functional.gelu(y_ref)
    elif act == "tanh":
        y_ref = torch.tanh(y_ref)
    if res:
        y_ref = y_ref + r.float()
    assert rel_err(y, y_ref) < 1e-2
    assert torch.isfinite(y.float()).all()


def test_device_sampler_semantics(dev):
    import numpy as np
    from fedrec_with_pytorchdistributed_amd.data.sampler import DeviceSampler
    from fedrec_with_pytorchdistributed_amd.data.synthetic import make_client_shards
    s = make_client_shards("tiny", 1)[0]
    arr = s.train
    ds = DeviceSampler(arr, 32, dev)
    cand, his = next(iter(ds.epoch(0)))
    assert cand.shape == (32, 5) and his.shape == (32, 50)
    rng = np.random.Generator(np.random.PCG64([0, 0, 0, 17]))
    order = rng.permutation(len(arr))[:32]
    c, h = cand.cpu().numpy(), his.cpu().numpy()
    for i, r in enumerate(order):
        negs = arr.negs(r)
        assert c[i, 0] == arr.pos[r]
        if len(negs) >= 4:
            picks = c[i, 1:].tolist()
            assert set(picks) <= set(negs.tolist())
        hh = arr.his(r)
        k = min(len(hh), 50)
        assert np.array_equal(h[i, :k], hh[-k:]) and np.all(h[i, k:] == 0)
    # distinct positions: sample from a list of distinct ids and check no repeats
    from fedrec_with_pytorchdistributed_amd.data.shard import ImpressionArrays
    a2 = ImpressionArrays(np.zeros(256, np.int32), np.arange(257, dtype=np.int64) * 6,
                          np.tile(np.arange(6, dtype=np.int32), 256), np.zeros(257, np.int64),
                          np.zeros(0, np.int32), np.zeros(256, np.int32))
    ds2 = DeviceSampler(a2, 256, dev, shuffle=False)
    c2, _ = next(iter(ds2.epoch(0)))
    c2 = c2.cpu().numpy()[:, 1:]
    assert all(len(set(r.tolist())) == 4 for r in c2)
    # every element is reachable and roughly uniform
    counts = np.bincount(c2.ravel(), minlength=6)
    assert counts.min() > 0.5 * counts.mean()


@pytest.mark.parametrize("variant", [1, 0])
@pytest.mark.parametrize("T", [50, 64, 9, 65, 200])
def test_title_attention_bwd(dev, T, variant):
    """variant 1 = persistent prefetching kernel (default), 0 = one-shot; n = 120 titles (1440 pairs > 1024
    persistent waves) so waves walk more than one (title, head) pair."""
    n, H, D = 120, 12, 768
    qkv = torch.randn(n * T, 3 * D, device=dev).to(torch.bfloat16)
    mask = (torch.rand(n, T, device=dev) < 0.7).to(torch.int32)
    mask[:, 0] = 1
    mask[1] = 0  # all-masked row
    dout = torch.randn(n * T, D, device=dev).to(torch.bfloat16)
    native.lib().title_attn_bwd_set_variant(variant)
    try:
        dq = native.lib().title_attention_bwd(qkv, dout, mask, H)
        assert torch.equal(native.lib().title_attention_bwd(qkv, dout, mask, H), dq)
    finally:
        native.lib().title_attn_bwd_set_variant(1)
    x = qkv.float().detach().requires_grad_(True)
    y = ref.title_attention(x, mask, H)
    y.backward(dout.float())
    ref_g = x.grad
    assert torch.isfinite(dq.float()).all()
    for part in range(3):
        a = dq.float()[:, part * D:(part + 1) * D]
        b = ref_g[:, part * D:(part + 1) * D]
        assert rel_err(a, b) < 3e-2, (part, rel_err(a, b))


def test_layer_norm_bwd(dev):
    x = (torch.randn(1000, 768, device=dev) * 2 + 0.5).to(torch.bfloat16)
    w = torch.randn(768, device=dev)
    dy = torch.randn(1000, 768, device=dev).to(torch.bfloat16)
    dx, dw, db = native.lib().layer_norm_bwd(x, w, dy, 1e-12)
    dx2, dw2, db2, dxs = native.lib().layer_norm_bwd_colsum(x, w, dy, 1e-12)
    assert torch.equal(dx2, dx) and rel_err(dw2, dw) < 1e-5 and rel_err(db2, db) < 1e-5
    assert rel_err(dxs, dx.float().sum(0)) < 1e-4  # fused bias gradient of the layer feeding the LN
    xf = x.float().requires_grad_(True)
    wf = w.clone().requires_grad_(True)
    bf = torch.zeros(768, device=dev, requires_grad=True)
    torch.nn.functional.layer_norm(xf, (768,), wf, bf, 1e-12).backward(dy.float())
    assert rel_err(dx, xf.grad) < 1e-2 and rel_err(dw, wf.grad) < 1e-3 and rel_err(db, bf.grad) < 1e-4


def test_layer_norm_bwd_drop(dev):
    """LN backward with the dropout backward of the layer that fed it (config-5 LN2 after the
    FFN dropout): dx as the plain kernel, dx o Z bit-equal to the separate dropout pass over
    dx, and the fused column sums are those of dx o Z (the lin2 bias gradient)."""
    x = (torch.randn(1000, 768, device=dev) * 2 + 0.5).to(torch.bfloat16)
    w = torch.randn(768, device=dev)
    dy = torch.randn(1000, 768, device=dev).to(torch.bfloat16)
    p, seed, off = 0.1, 99, 5
    dx, dw, db = native.lib().layer_norm_bwd(x, w, dy, 1e-12)
    dx2, dxz, dw2, db2, cs = native.lib().layer_norm_bwd_drop(x, w, dy, 1e-12, p, seed, off)
    assert torch.equal(dx2, dx) and rel_err(dw2, dw) < 1e-5 and rel_err(db2, db) < 1e-5
    assert torch.equal(dxz, ops.dropout_add(dx, None, p, seed, off))
    assert rel_err(cs, dxz.float().sum(0)) < 1e-4
    kept = float((dxz != 0).float().mean() / (dx != 0).float().mean())
    assert 0.87 < kept < 0.93


def test_multi_cast(dev):
    """One-launch refresh of compute copies: fp32 masters -> bf16 (or fp32) destinations,
    including slices of a fused destination, equal to .to(bf16) element for element."""
    srcs = [torch.randn(768, 768, device=dev), torch.randn(768, device=dev), torch.randn(3072, 768, device=dev),
            torch.randn(1000, 8, device=dev)]
    fused = torch.empty(2 * 768, 768, device=dev, dtype=torch.bfloat16)
    dsts = [fused[:768], torch.empty(768, device=dev), torch.empty(3072, 768, device=dev, dtype=torch.bfloat16),
            fused[768:].view(-1)[:8000].view(1000, 8)]
    assert native.lib().multi_cast(srcs, dsts)
    for a, b in zip(srcs, dsts):
        assert torch.equal(b, a.to(b.dtype))
    many_s = [torch.randn(64, device=dev) for _ in range(130)]  # > 96 segments: several launches
    many_d = [torch.empty(64, device=dev, dtype=torch.bfloat16) for _ in range(130)]
    assert native.lib().multi_cast(many_s, many_d)
    assert all(torch.equal(b, a.to(torch.bfloat16)) for a, b in zip(many_s, many_d))
    # the optional step-counter bump: +1 per call, however many launches the call takes
    ctr = torch.full((1,), 41, device=dev, dtype=torch.int64)
    assert native.lib().multi_cast(many_s, many_d, ctr)
    assert native.lib().multi_cast(srcs, dsts, ctr)
    assert int(ctr.item()) == 43
    # ragged sizes and 4-byte-aligned slices take the element path
    odd_s = [torch.randn(13, device=dev), torch.randn(1, device=dev), torch.randn(1001, device=dev)[1:]]
    odd_d = [torch.empty(13, device=dev), torch.empty(3, device=dev, dtype=torch.bfloat16)[1:2],
             torch.empty(1000, device=dev)]
    assert native.lib().multi_cast(odd_s, odd_d)
    assert all(torch.equal(b, a.to(b.dtype)) for a, b in zip(odd_s, odd_d))


def test_multi_cast_transposed_views(dev):
    """Transposed bf16 views as cast destinations (the register-direct GEMMs' W^T copies): ragged
    R / C, side by side in one stacked matrix, beside plain segments of the same launch, and
    through copy_cast (a step graph's input launch)."""
    ws = [torch.randn(400, 400, device=dev), torch.randn(200, 400, device=dev), torch.randn(37, 130, device=dev)]
    stack = torch.full((400, 600), 7.0, device=dev, dtype=torch.bfloat16)
    odd = torch.empty(130, 40, device=dev, dtype=torch.bfloat16)
    plain_s, plain_d = torch.randn(1000, device=dev), torch.empty(1000, device=dev, dtype=torch.bfloat16)
    dsts = [stack[:, :400].t(), stack[:, 400:].t(), odd[:, :37].t()]
    assert native.lib().multi_cast([plain_s] + ws, [plain_d] + dsts)
    assert torch.equal(plain_d, plain_s.to(torch.bfloat16))
    assert torch.equal(stack[:, :400], ws[0].t().to(torch.bfloat16))
    assert torch.equal(stack[:, 400:], ws[1].t().to(torch.bfloat16))
    assert torch.equal(odd[:, :37], ws[2].t().to(torch.bfloat16))
    stack.fill_(0)
    a, b = torch.arange(10, device=dev, dtype=torch.int32), torch.empty(16, device=dev, dtype=torch.int32)
    assert native.lib().copy_cast([a], [b], [-1], [plain_s] + ws[:2], [plain_d] + dsts[:2], None, None)
    assert torch.equal(b[:10], a) and bool((b[10:] == -1).all())
    assert torch.equal(stack[:, :400], ws[0].t().to(torch.bfloat16))
    assert torch.equal(stack[:, 400:], ws[1].t().to(torch.bfloat16))


@pytest.mark.gpu
def test_copy_cast(dev):
    """A step graph's input launch: int32 batch copies whose destinations are padded with a fill
    word (bit patterns kept: negative ids look like NaN floats), empty sources (fill only),
    weight casts to bf16 / fp32 and both counter bumps -- one launch, equal to the separate ops."""
    g = torch.Generator(device="cpu").manual_seed(3)
    cand = torch.randint(-5, 65000, (64, 5), generator=g, dtype=torch.int32).to(dev)
    ptr = torch.arange(0, 1601 * 3, 3, dtype=torch.int32).to(dev)
    odd = torch.randint(-(2 ** 31), 2 ** 31 - 1, (37,), generator=g, dtype=torch.int64).to(torch.int32).to(dev)
    none = torch.empty(0, dtype=torch.int32, device=dev)
    c_dst = torch.full((64, 5), 7, dtype=torch.int32, device=dev)
    p_dst = torch.full((1793,), 7, dtype=torch.int32, device=dev)
    o_dst = torch.full((41,), 7, dtype=torch.int32, device=dev)
    n_dst = torch.full((1,), 7, dtype=torch.int32, device=dev)
    w = torch.randn(384, 768, device=dev)
    b = torch.randn(1200, device=dev)
    wb = torch.empty(384, 768, device=dev, dtype=torch.bfloat16)
    bf = torch.empty(1200, device=dev)
    c1 = torch.full((1,), 10, device=dev, dtype=torch.int64)
    c2 = torch.full((1,), 20, device=dev, dtype=torch.int64)
    assert native.lib().copy_cast([cand, ptr, odd[1:], none], [c_dst, p_dst, o_dst, n_dst], [0, 4800, -1, 1565],
                                  [w, b], [wb, bf], c1, c2)
    assert torch.equal(c_dst, cand)
    assert torch.equal(p_dst[:1601], ptr) and bool((p_dst[1601:] == 4800).all())
    assert torch.equal(o_dst[:36], odd[1:]) and bool((o_dst[36:] == -1).all())
    assert int(n_dst.item()) == 1565
    assert torch.equal(wb, w.to(torch.bfloat16)) and torch.equal(bf, b)
    assert int(c1.item()) == 11 and int(c2.item()) == 21
    # no casts: copies alone, no bumps
    assert native.lib().copy_cast([cand], [c_dst], [0], [], [], None, None)
    # transposed: [R, C] fp32 -> bf16 [C, R] views, side by side in a fused [C, 3R] destination
    ws = [torch.randn(768, 768, device=dev) for _ in range(3)] + [torch.randn(3072, 768, device=dev)]
    fused_t = torch.empty(768, 3 * 768, device=dev, dtype=torch.bfloat16)
    w1t = torch.empty(768, 3072, device=dev, dtype=torch.bfloat16)
    dt = [fused_t[:, i * 768:(i + 1) * 768] for i in range(3)] + [w1t]
    assert native.lib().multi_cast_t(ws, dt)
    assert torch.equal(fused_t, torch.cat(ws[:3], 0).to(torch.bfloat16).t())
    assert torch.equal(w1t, ws[3].to(torch.bfloat16).t())


def test_gelu_fwd_bwd(dev):
    z = (torch.randn(4096, device=dev) * 3).to(torch.bfloat16)
    dh = torch.randn(4096, device=dev).to(torch.bfloat16)
    h = native.lib().gelu(z, None)
    dz = native.lib().gelu(z, dh)
    zf = z.float().requires_grad_(True)
    hf = torch.nn.functional.gelu(zf)
    hf.backward(dh.float())
    assert rel_err(h, hf) < 5e-3 and rel_err(dz, zf.grad) < 5e-3


@pytest.mark.parametrize("M,N", [(78850, 768), (5000, 3072), (3, 2304), (1001, 38400)])
def test_colsum(dev, M, N):
    x = torch.randn(M, N, device=dev).to(torch.bfloat16)
    got = native.lib().colsum(x)
    want = x.float().sum(0)
    assert rel_err(got, want) < 1e-5
    if N % 3 == 0 and (N // 3) % 8 == 0:  # a column slice (the Q third of a [M, 3D] gradient)
        sl = x[:, : N // 3]
        assert rel_err(native.lib().colsum(sl), sl.float().sum(0)) < 1e-5


def test_embed_grad(dev):
    """Sort-based word-embedding gradient == index_add with the pad row zeroed."""
    R, D, V = 20000, 768, 3000
    tok = torch.randint(0, V, (R,), device=dev, dtype=torch.int32)
    tok[::3] = 0  # lots of pad tokens
    tok[:500] = 101  # a heavy [CLS]-like token
    dx = torch.randn(R, D, device=dev).to(torch.bfloat16)
    srt, perm = torch.sort(tok, stable=True)
    got = native.lib().embed_grad(dx, srt.to(torch.int32), perm.to(torch.int32), V)
    want = torch.zeros(V, D, device=dev).index_add_(0, tok.long(), dx.float())
    want[0] = 0
    got[0] = 0
    assert rel_err(got, want) < 1e-5


@pytest.mark.parametrize("M", [78850, 5000, 300])
def test_linear_gelu_dual(dev, M):
    """Training FFN1: the dual-store GEMM gives z = x w^T + b and GELU(z) in one pass (the
    300-row case takes the GEMM + GELU fallback)."""
    K, N = 768, 3072
    x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    lib = native.lib()
    h, z = lib.linear_gelu_dual(x, w, b)
    z_ref = lib.linear(x, w, b, 0, None)
    h_ref = lib.linear(x, w, b, 1, None)
    assert torch.equal(z, z_ref)
    assert rel_err(h, h_ref) < 5e-3
    sl = slice(0, min(M, 1024))
    assert rel_err(h[sl], torch.nn.functional.gelu(x[sl].float() @ w.float().t() + b)) < 1e-2


def test_backbone_long_titles_match_reference(dev):
    """A 2-layer DistilBERT-width backbone on 96-token titles (T > 64: unpacked path, long
    attention kernels) against the fp32 eager oracle with the same weights."""
    from fedrec_with_pytorchdistributed_amd.config import BackboneConfig
    from fedrec_with_pytorchdistributed_amd.models.backbone import Backbone

    torch.manual_seed(0)
    bb = Backbone(BackboneConfig(name="distilbert-2l", n_layers=2)).to(dev)
    n, T = 6, 96
    tok = torch.randint(1000, 29000, (n, T), device=dev, dtype=torch.int32)
    lens = torch.tensor([96, 70, 65, 20, 3, 0])
    mask = (torch.arange(T)[None, :] < lens[:, None]).to(torch.int32).to(dev)
    tok = tok * mask
    y = bb.forward(tok, mask, torch.bfloat16)
    P = bb.compute_weights(torch.float32)
    y_ref = ref.backbone_forward(tok.long(), mask, P, 2, 12, bb.cfg.ln_eps)
    assert torch.isfinite(y.float()).all()
    assert rel_err(y, y_ref) < 2e-2


@pytest.mark.parametrize("variant", [-1, 0, 6, 9])
@pytest.mark.parametrize("M", [300, 9000])
def test_gemm_gelu_bwd_epilogue(dev, variant, M):
    """act = 3 (training FFN2 dgrad): C = (A W^T) * GELU'(R) with R = the saved pre-activation,
    every GEMM variant, against the fp32 product times autograd's exact-erf GELU derivative."""
    N, K = 3072, 768
    g = torch.Generator(device="cpu").manual_seed(M + variant)
    a = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev, torch.bfloat16)
    z = (torch.randn(M, N, generator=g) * 2).to(dev, torch.bfloat16)
    lib = native.lib()
    lib.gemm_set_variant(variant)
    try:
        y = lib.linear(a, w, None, 3, z)
    finally:
        lib.gemm_set_variant(-1)
    zf = z.float().requires_grad_(True)
    torch.nn.functional.gelu(zf).backward(torch.ones_like(zf))
    ref_y = (a.float() @ w.float().t()) * zf.grad
    assert torch.isfinite(y.float()).all()
    assert rel_err(y, ref_y) < 1e-2


@pytest.mark.parametrize("M", [300, 9000, 78850])
def test_linear_gelu_bwd_with_colsum(dev, M):
    """Training FFN2 dgrad op: dz = (dh W^T) * GELU'(z) plus the FFN1 bias gradient (column sums
    of dz) from the same GEMM pass; small M falls back to the plain kernels (colsum None)."""
    N, K = 3072, 768
    g = torch.Generator(device="cpu").manual_seed(M)
    a = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev, torch.bfloat16)
    z = (torch.randn(M, N, generator=g) * 2).to(dev, torch.bfloat16)
    lib = native.lib()
    dz, cs = lib.linear_gelu_bwd(a, w, z)
    assert torch.equal(dz, lib.linear(a, w, None, 3, z))
    if M >= 4096:
        assert cs is not None
        assert rel_err(cs, dz.float().sum(0)) < 2e-3
        dz2, cs2 = lib.linear_gelu_bwd(a, w, z)
        assert torch.equal(cs2, cs)  # deterministic partials + fixed-order sum
    else:
        assert cs is None


@pytest.mark.parametrize("M,N", [(78850, 3072), (300, 3072), (5, 64)])
def test_gelu_bwd_colsum(dev, M, N):
    """Streaming training-FFN1 backward: dz = dF * GELU'(z) (exact-erf autograd reference) and
    its column sums (the FFN1 bias gradient), deterministic."""
    g = torch.Generator(device="cpu").manual_seed(M + N)
    df = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    z = (torch.randn(M, N, generator=g) * 2).to(dev, torch.bfloat16)
    dz, cs = native.lib().gelu_bwd_colsum(df, z)
    zf = z.float().requires_grad_(True)
    torch.nn.functional.gelu(zf).backward(df.float())
    assert rel_err(dz, zf.grad) < 5e-3
    assert rel_err(cs, dz.float().sum(0)) < 1e-5
    dz2, cs2 = native.lib().gelu_bwd_colsum(df, z)
    assert torch.equal(dz2, dz) and torch.equal(cs2, cs)


def test_device_ops_refuse_non_bf16(dev):
    """A device tensor of a dtype without a kernel raises instead of running torch eager."""
    from fedrec_with_pytorchdistributed_amd import ops as O
    x = torch.randn(256, 768, device=dev)
    w = torch.randn(384, 768, device=dev)
    with pytest.raises(RuntimeError, match="no HIP kernel"):
        O.linear(x, w)
    with pytest.raises(RuntimeError, match="no HIP kernel"):
        O.layer_norm(x, torch.ones(768, device=dev), torch.zeros(768, device=dev), 1e-12)



def test_adam_dev_skips_on_status_word(dev):
    """The in-graph Adam with the gradient all-reduce's status word: nonzero (a peer timed out,
    the sum was poisoned) -> no update of p / m / v and the step's loss slot is NaN; zero -> the
    ordinary step, equal to the eager fused Adam."""
    n = 1024
    lib = native.lib()
    g = torch.Generator(device="cpu").manual_seed(0)
    p0 = torch.randn(n, generator=g).to(dev)
    gr = torch.randn(n, generator=g).to(dev)
    step = torch.ones(1, dtype=torch.int64, device=dev)
    loss = torch.full((1,), 1.5, device=dev)
    for flag in (1, 0):
        p, m, v = p0.clone(), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        ring = torch.zeros(8, device=dev)
        skip = torch.full((1,), flag, dtype=torch.int32, device=dev)
        lib.adam_dev(p, gr.clone(), m, v, step, loss, ring, 1e-3, 0.9, 0.999, 1e-8, 0.5, None, None, skip)
        torch.cuda.synchronize()
        if flag:
            assert torch.equal(p, p0) and not bool(m.any()) and not bool(v.any())
            assert torch.isnan(ring[0])
        else:
            pe, me, ve = p0.clone(), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
            ops.adam_flat(pe, gr.clone(), me, ve, 1, 1e-3, 0.9, 0.999, 1e-8, 0.5)
            assert torch.allclose(p, pe, atol=1e-7) and float(ring[0]) == 1.5
