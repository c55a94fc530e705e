"""Weight-gradient TN GEMM (csrc/gemm_wgrad.hip) against an fp32 torch reference of the same
bf16 operands: dW = dy^T x over a long reduction dim, partial tiles in every dimension."""
import pytest
import torch

from fedrec_with_pytorchdistributed_amd.ops import functional as OF
from fedrec_with_pytorchdistributed_amd.ops import native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(78260, 2304, 768), (4113, 768, 3072), (50, 384, 768), (1000, 200, 400),
                                   (80000, 384, 768), (64, 256, 256), (129, 8, 16), (3000, 1200, 400)])
def test_wgrad_matches_fp32(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    out = native.lib().wgrad(dy, x)
    ref = dy.double().t() @ x.double()
    assert out.dtype == torch.float32 and out.shape == (N, K)
    err = (out.double() - ref).abs().max().item()
    scale = (dy.double().abs().t() @ x.double().abs()).max().item()
    assert err <= 1e-5 * scale + 1e-4, (err, scale)


def test_wgrad_deterministic_and_wired():
    g = torch.Generator(device="cuda").manual_seed(7)
    dy = torch.randn(20000, 768, device="cuda", generator=g).bfloat16()
    x = torch.randn(20000, 768, device="cuda", generator=g).bfloat16()
    a = native.lib().wgrad(dy, x)
    b = native.lib().wgrad(dy, x)
    assert torch.equal(a, b)
    assert torch.equal(OF.wgrad(dy, x), a)  # the training path runs this kernel


def test_wgrad_zero_rows():
    dy = torch.zeros(0, 256, device="cuda", dtype=torch.bfloat16)
    x = torch.zeros(0, 128, device="cuda", dtype=torch.bfloat16)
    assert torch.count_nonzero(native.lib().wgrad(dy, x)) == 0
