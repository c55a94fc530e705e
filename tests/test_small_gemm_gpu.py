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


def _check(g, tol=2e-3):
    want = ops.small_gemm_ref(g)
    ops.small_gemm(g)
    got = g.C.reshape(-1)[: g.M * g.ldc].view(g.M, g.ldc)[:, : g.N]
    assert _rel(got, want) < tol, _rel(got, want)


def test_nt_gather_dropout_bias_tanh(dev):
    torch.manual_seed(0)
    x = torch.randn(900, 400, device=dev)
    gidx = torch.randint(0, 900, (3200,), device=dev, dtype=torch.int32)
    w = torch.randn(200, 400, device=dev) * 0.05
    b = torch.randn(200, device=dev)
    C = torch.zeros(3200, 200, device=dev)
    _check(Gemm(x, w, C, 3200, 200, 400, 400, 400, 200, bias=b, act=1, gidx=gidx, gather_on=1,
                pdrop=0.2, drop_on=1, drop_ld=400, seed=5, offset=9))


def test_tn_wgrad_with_gathered_dropped_input(dev):
    torch.manual_seed(1)
    dy = torch.randn(3200, 1200, device=dev)  # stored [K, M]: dY, column slice = one projection
    x = torch.randn(700, 400, device=dev)
    gidx = torch.randint(0, 700, (3200,), device=dev, dtype=torch.int32)
    C = torch.zeros(400, 400, device=dev)
    _check(Gemm(dy[:, 400:], x, C, 400, 400, 3200, 1200, 400, 400, a_mode=1, b_mode=1, gidx=gidx, gather_on=2,
                pdrop=0.2, drop_on=2, drop_ld=400, seed=3, offset=4))


def test_nn_dgrad_dropout_epilogue_accumulate(dev):
    torch.manual_seed(2)
    dy = torch.randn(3200, 400, device=dev)
    w = torch.randn(400, 400, device=dev) * 0.05
    C = torch.randn(3200, 400, device=dev)
    _check(Gemm(dy, w, C, 3200, 400, 400, 400, 400, 400, b_mode=1, accumulate=True, pdrop=0.2, drop_on=3,
                drop_ld=400, seed=1, offset=2))


def test_grouped_launch_and_odd_shapes(dev):
    torch.manual_seed(3)
    gs, wants = [], []
    for (M, N, K) in ((17, 33, 5), (64, 64, 64), (1565, 400, 768), (3, 200, 1200)):
        A = torch.randn(M, K, device=dev)
        B = torch.randn(N, K, device=dev)
        C = torch.zeros(M, N, device=dev)
        g = Gemm(A, B, C, M, N, K, K, K, N, alpha=0.5)
        gs.append(g)
        wants.append(ops.small_gemm_ref(g))
    ops.small_gemm(*gs)
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


def test_k_segmented_b_with_dropout_epilogue(dev):
    """dx = [dQ|dK|dV] [Wq; Wk; Wv]: one GEMM over three separately stored weight blocks."""
    torch.manual_seed(5)
    dq = torch.randn(3200, 1200, device=dev)
    ws = [torch.randn(400, 400, device=dev) * 0.05 for _ in range(3)]
    C = torch.zeros(3200, 400, device=dev)
    _check(Gemm(dq, ws[0], C, 3200, 400, 1200, 1200, 400, 400, b_mode=1, bseg=(ws[1], ws[2]), kseg=400,
                pdrop=0.2, drop_on=3, drop_ld=400, seed=2, offset=3))
