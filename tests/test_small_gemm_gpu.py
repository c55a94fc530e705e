"""csrc/small_gemm.hip against an fp32 torch emulation (operands rounded to bf16 as the kernel
does): every layout, the fused row gather / Philox dropout prologues, the dropout epilogue,
bias / tanh / accumulate, and several GEMMs per launch; plus the deterministic fp32 colsum."""

import pytest
import torch

from fedrec_with_pytorchdistributed_amd import ops
from fedrec_with_pytorchdistributed_amd.ops import Gemm

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


TILES = [1, 2, 3, 4]  # 64x64, 128x64, 64x128, 128x128


def _check(g, tol=2e-3, tile=0):
    want = ops.small_gemm_ref(g)
    ops.small_gemm(g, tile=tile)
    got = g.C.reshape(-1)[: g.M * g.ldc].view(g.M, g.ldc)[:, : g.N]
    assert _rel(got, want) < tol, _rel(got, want)


@pytest.mark.parametrize("tile", TILES)
def test_nt_gather_dropout_bias_tanh(dev, tile):
    torch.manual_seed(0)
    x = torch.randn(900, 400, device=dev)
    gidx = torch.randint(0, 900, (3200,), device=dev, dtype=torch.int32)
    w = torch.randn(200, 400, device=dev) * 0.05
    b = torch.randn(200, device=dev)
    C = torch.zeros(3200, 200, device=dev)
    _check(Gemm(x, w, C, 3200, 200, 400, 400, 400, 200, bias=b, act=1, gidx=gidx, gather_on=1,
                pdrop=0.2, drop_on=1, drop_ld=400, seed=5, offset=9), tile=tile)


@pytest.mark.parametrize("tile", TILES)
def test_tn_wgrad_with_gathered_dropped_input(dev, tile):
    torch.manual_seed(1)
    dy = torch.randn(3200, 1200, device=dev)  # stored [K, M]: dY, column slice = one projection
    x = torch.randn(700, 400, device=dev)
    gidx = torch.randint(0, 700, (3200,), device=dev, dtype=torch.int32)
    C = torch.zeros(400, 400, device=dev)
    _check(Gemm(dy[:, 400:], x, C, 400, 400, 3200, 1200, 400, 400, a_mode=1, b_mode=1, gidx=gidx, gather_on=2,
                pdrop=0.2, drop_on=2, drop_ld=400, seed=3, offset=4), tile=tile)


@pytest.mark.parametrize("tile", TILES)
def test_nn_dgrad_dropout_epilogue_accumulate(dev, tile):
    torch.manual_seed(2)
    dy = torch.randn(3200, 400, device=dev)
    w = torch.randn(400, 400, device=dev) * 0.05
    C = torch.randn(3200, 400, device=dev)
    _check(Gemm(dy, w, C, 3200, 400, 400, 400, 400, 400, b_mode=1, accumulate=True, pdrop=0.2, drop_on=3,
                drop_ld=400, seed=1, offset=2), tile=tile)


@pytest.mark.parametrize("tile", [0] + TILES)
def test_grouped_launch_and_odd_shapes(dev, tile):
    torch.manual_seed(3)
    gs, wants = [], []
    for (M, N, K) in ((17, 33, 5), (64, 64, 64), (1565, 400, 768), (3, 200, 1200)):
        A = torch.randn(M, K, device=dev)
        B = torch.randn(N, K, device=dev)
        C = torch.zeros(M, N, device=dev)
        g = Gemm(A, B, C, M, N, K, K, K, N, alpha=0.5)
        gs.append(g)
        wants.append(ops.small_gemm_ref(g))
    ops.small_gemm(*gs, tile=tile)
    for g, w in zip(gs, wants):
        assert _rel(g.C, w) < 2e-3


def test_colsum_f32_deterministic(dev):
    torch.manual_seed(4)
    X = torch.randn(3200, 1200, device=dev)
    Y = torch.randn(64, 200, device=dev)
    o1 = torch.zeros(400, device=dev)
    o2 = torch.zeros(200, device=dev)
    ops.colsum_f32([(X[:, 400:], o1, 3200, 400, 1200), (Y, o2, 64, 200, 200)])
    assert torch.allclose(o1, X[:, 400:800].sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(o2, Y.sum(0), rtol=1e-4, atol=1e-4)
    o3 = torch.zeros(400, device=dev)
    ops.colsum_f32([(X[:, 400:], o3, 3200, 400, 1200)])
    assert torch.equal(o1, o3)


@pytest.mark.parametrize("tile", TILES)
def test_k_segmented_b_with_dropout_epilogue(dev, tile):
    """dx = [dQ|dK|dV] [Wq; Wk; Wv]: one GEMM over three separately stored weight blocks."""
    torch.manual_seed(5)
    dq = torch.randn(3200, 1200, device=dev)
    ws = [torch.randn(400, 400, device=dev) * 0.05 for _ in range(3)]
    C = torch.zeros(3200, 400, device=dev)
    _check(Gemm(dq, ws[0], C, 3200, 400, 1200, 1200, 400, 400, b_mode=1, bseg=(ws[1], ws[2]), kseg=400,
                pdrop=0.2, drop_on=3, drop_ld=400, seed=2, offset=3), tile=tile)


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("a_mode,b_mode", [(0, 0), (0, 1), (1, 1)])
@pytest.mark.parametrize("dt", ["a", "b", "ab"])
def test_bf16_operands_match_fp32_operands_bitwise(dev, tile, a_mode, b_mode, dt):
    """A bf16 operand is what the kernel's fp32 loads round to: the product is bitwise the one
    of the fp32 operand (same tile, same order), for every layout and tile."""
    torch.manual_seed(6)
    M, N, K = 1000, 300, 456
    A = torch.randn(M, K, device=dev) if a_mode == 0 else torch.randn(K, M, device=dev)
    B = torch.randn(N, K, device=dev) if b_mode == 0 else torch.randn(K, N, device=dev)
    bias = torch.randn(N, device=dev)
    lda, ldb = (K if a_mode == 0 else M), (K if b_mode == 0 else N)
    C32 = torch.zeros(M, N, device=dev)
    ops.small_gemm(Gemm(A, B, C32, M, N, K, lda, ldb, N, a_mode=a_mode, b_mode=b_mode, bias=bias, act=1), tile=tile)
    Ah = A.to(torch.bfloat16) if "a" in dt else A
    Bh = B.to(torch.bfloat16) if "b" in dt else B
    C16 = torch.zeros(M, N, device=dev)
    g = Gemm(Ah, Bh, C16, M, N, K, lda, ldb, N, a_mode=a_mode, b_mode=b_mode, bias=bias, act=1)
    ops.small_gemm(g, tile=tile)
    assert torch.equal(C32, C16)
    assert _rel(C16, ops.small_gemm_ref(g)) < 2e-3


@pytest.mark.parametrize("tile", TILES)
def test_bf16_unaligned_and_odd_edges(dev, tile):
    """bf16 operands whose rows are not 16-byte aligned (odd K / odd offsets): the scalar
    edge path, every element once."""
    torch.manual_seed(7)
    M, N, K = 77, 45, 131
    A = torch.randn(M * K + 1, device=dev).to(torch.bfloat16)[1:].view(M, K)
    B = torch.randn(K, N, device=dev).to(torch.bfloat16)
    C = torch.zeros(M, N, device=dev)
    _check(Gemm(A, B, C, M, N, K, K, N, N, b_mode=1), tile=tile)


def test_gather_dropout_bf16_is_rounded_fp32(dev):
    torch.manual_seed(8)
    v = torch.randn(500, 400, device=dev)
    idx = torch.randint(0, 500, (3200,), device=dev, dtype=torch.int32)
    off = torch.tensor([7], device=dev, dtype=torch.int64)
    x32 = ops.gather_dropout(v, idx, 0.2, 11, 3, off)
    x16 = ops.gather_dropout(v, idx, 0.2, 11, 3, off, bf16_out=True)
    assert x16.dtype == torch.bfloat16 and torch.equal(x16, x32.to(torch.bfloat16))


def test_colsum_f32_scalar_and_vector_paths(dev):
    torch.manual_seed(9)
    X = torch.randn(3201, 1204, device=dev)
    Z = torch.randn(3201, 1203, device=dev)
    outs = [torch.zeros(n, device=dev) for n in (33, 400, 1203)]
    # a misaligned view (scalar path), an aligned float4 view, and an odd-width matrix (scalar)
    ops.colsum_f32([(X[:, 1:], outs[0], 3201, 33, 1204), (X[:, 400:], outs[1], 3200, 400, 1204),
                    (Z, outs[2], 3201, 1203, 1203)])
    assert torch.allclose(outs[0], X[:, 1:34].sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(outs[1], X[:3200, 400:800].sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(outs[2], Z.sum(0), rtol=1e-4, atol=1e-3)
    Y = torch.randn(4096, 800, device=dev)
    o = torch.zeros(800, device=dev)
    ops.colsum_f32([(Y, o, 4096, 800, 800)])
    assert torch.allclose(o, Y.double().sum(0).float(), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("ah", [False, True])
def test_asum_column_sums_of_a(dev, tile, ah):
    """asum (a_mode 1): the fp32 column sums of the stored-transposed A -- a weight gradient's
    bias gradient -- from the same launch, split-K and not, next to a second desc."""
    torch.manual_seed(10)
    outs = []
    gs = []
    for (M, N, K) in ((1200, 400, 3200), (200, 400, 3200), (400, 768, 1664), (72, 40, 300)):
        A = torch.randn(K, M, device=dev)
        if ah:
            A = A.to(torch.bfloat16)
        Bm = torch.randn(K, N, device=dev).to(torch.bfloat16)
        C = torch.zeros(M, N, device=dev)
        a_s = torch.full((M,), float("nan"), device=dev)
        gs.append(Gemm(A, Bm, C, M, N, K, M, N, N, a_mode=1, b_mode=1, asum=a_s))
        outs.append((A, a_s, ops.small_gemm_ref(gs[-1])))
    ops.small_gemm(gs[0], gs[1], tile=tile)
    ops.small_gemm(gs[2], gs[3], tile=tile)
    for g, (A, a_s, want) in zip(gs, outs):
        assert _rel(g.C, want) < 2e-3
        ref = A.double().sum(0)
        assert torch.allclose(a_s.double(), ref, rtol=1e-5, atol=1e-3), float((a_s.double() - ref).abs().max())


@pytest.mark.parametrize("MNK", [(3200, 1200, 400), (1565, 400, 768), (77, 45, 136), (64, 64, 64), (3, 200, 1200),
                                 (200, 400, 3200), (5000, 72, 8)])
def test_dma_ring_matches_register_queue_bitwise(dev, MNK):
    """bf16 x bf16 k-contiguous launches take the LDS-DMA ring (tile 0 / 1); tile 5 forces the
    register-queue 64 x 64 kernel: same tiles, same k order -> bitwise equal C, with row / column
    / k tails, split-K partials, bias + tanh, the dropout epilogue and accumulate."""
    torch.manual_seed(11)
    M, N, K = MNK
    A = (torch.randn(M, K + 8, device=dev)).to(torch.bfloat16)  # ld > K: a strided view of rows
    B = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    C0 = torch.randn(M, N, device=dev)
    kw = dict(bias=bias, act=1) if K < 1000 else dict(accumulate=True, pdrop=0.2, drop_on=3, drop_ld=N - N % 16 + 16,
                                                     seed=4, offset=5)
    outs = []
    for tile in (5, 0, 1):
        C = C0.clone()
        g = Gemm(A, B, C, M, N, K, K + 8, K, N, **kw)
        if tile == 5:
            want = ops.small_gemm_ref(g)
        ops.small_gemm(g, tile=tile)
        outs.append(C)
    assert _rel(outs[0], want) < 2e-3
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("a_mode,b_mode", [(0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("MNK", [(3200, 400, 1200), (1200, 400, 3200), (72, 40, 300), (400, 768, 1568)])
def test_dma_ring_transposed_operands_and_asum(dev, a_mode, b_mode, MNK):
    """The DMA ring with stored-transposed operands (ds_read_b64_tr_b16 fragments) is bitwise the
    register-queue kernel (tile 5), split-K or not; a transposed A's column sums (asum) come from
    the ring's ones-MFMA and match a float64 sum of the same bf16 values."""
    torch.manual_seed(12)
    M, N, K = MNK
    A = (torch.randn(M, K, device=dev) if a_mode == 0 else torch.randn(K, M, device=dev)).to(torch.bfloat16)
    B = (torch.randn(N, K, device=dev) if b_mode == 0 else torch.randn(K, N, device=dev)).to(torch.bfloat16)
    lda, ldb = (K if a_mode == 0 else M), (K if b_mode == 0 else N)
    outs, sums = [], []
    for tile in (5, 0):
        C = torch.zeros(M, N, device=dev)
        s = torch.full((M,), float("nan"), device=dev) if a_mode == 1 else None
        g = Gemm(A, B, C, M, N, K, lda, ldb, N, a_mode=a_mode, b_mode=b_mode, asum=s)
        if tile == 5:
            want = ops.small_gemm_ref(g)
        ops.small_gemm(g, tile=tile)
        outs.append(C)
        sums.append(s)
    assert _rel(outs[1], want) < 2e-3
    assert torch.equal(outs[0], outs[1])
    if a_mode == 1:
        ref = A.double().sum(0)
        assert torch.allclose(sums[1].double(), ref, rtol=1e-5, atol=1e-3), float((sums[1].double() - ref).abs().max())


# register-direct form (tile codes 1000 + 10 f + P, + 100 with split-K): bf16 B [N, K], bf16 or
# fp32 A [M, K], the epilogue options of the step's launches, ragged M / N / K
RD = [1002, 1003, 1004, 1012, 1013, 1023, 1033, 1103]


@pytest.mark.parametrize("tile", RD)
def test_rd_nt_bias_tanh(dev, tile):
    torch.manual_seed(7)
    a = torch.randn(3190, 392, device=dev).to(torch.bfloat16)
    w = (torch.randn(203, 392, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(203, device=dev)
    C = torch.zeros(3190, 203, device=dev)
    _check(Gemm(a, w, C, 3190, 203, 392, 392, 392, 203, bias=b, act=1), tile=tile)


@pytest.mark.parametrize("tile", RD)
def test_rd_dgrad_dropout_accumulate_strided_b(dev, tile):
    torch.manual_seed(8)
    dy = torch.randn(3200, 1200, device=dev).to(torch.bfloat16)
    wt = (torch.randn(400, 1400, device=dev) * 0.05).to(torch.bfloat16)  # [W^T | more]: ldb 1400
    C = torch.randn(3200, 400, device=dev)
    _check(Gemm(dy, wt, C, 3200, 400, 1200, 1200, 1400, 400, accumulate=True, pdrop=0.2, drop_on=3, drop_ld=400,
                seed=4, offset=6), tile=tile)
    _check(Gemm(dy[:, :200], wt[:, 1200:], C, 3200, 400, 200, 1200, 1400, 400, accumulate=True), tile=tile)


@pytest.mark.parametrize("tile", [1002, 1032, 1033])
def test_rd_fp32_a(dev, tile):
    torch.manual_seed(9)
    dy = torch.randn(1565, 400, device=dev)
    wt = (torch.randn(768, 400, device=dev) * 0.05).to(torch.bfloat16)
    C = torch.zeros(1565, 768, device=dev)
    _check(Gemm(dy, wt, C, 1565, 768, 400, 400, 400, 768), tile=tile)


def test_rd_matches_lds_form_bitwise(dev):
    """Same operands, same k order, same fp32 MFMA accumulation: the register-direct C equals the
    LDS-DMA ring's bit for bit (the two forms are interchangeable per launch)."""
    torch.manual_seed(10)
    a = torch.randn(3200, 400, device=dev).to(torch.bfloat16)
    w = (torch.randn(200, 400, device=dev) * 0.05).to(torch.bfloat16)
    c1, c2 = torch.zeros(3200, 200, device=dev), torch.zeros(3200, 200, device=dev)
    ops.small_gemm(Gemm(a, w, c1, 3200, 200, 400, 400, 400, 200), tile=1)
    ops.small_gemm(Gemm(a, w, c2, 3200, 200, 400, 400, 400, 200), tile=1003)
    assert torch.equal(c1, c2)
