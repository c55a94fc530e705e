"""The ping-pong NT GEMM on column counts that are not a multiple of its 256-wide tile (the
text head's att_fc1, N = 384): partial last column tile, against an fp32 torch reference."""
import pytest
import torch

from fedrec_with_pytorchdistributed_amd.ops import native

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _variant9():
    native.lib().gemm_set_variant(9)  # the partial-tile path is opt-in (slower at N = 384 in the step)
    yield
    native.lib().gemm_set_variant(-1)


@pytest.mark.parametrize("M,N,K,act", [(80000, 384, 768, 2), (5000, 640, 768, 0), (4100, 384, 256, 1),
                                       (78850, 384, 768, 0)])
def test_linear_partial_tile(M, N, K, act):
    g = torch.Generator(device="cuda").manual_seed(N + K)
    x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    y = native.lib().linear(x, w, b, act, None)
    ref = x.float() @ w.float().t() + b
    ref = {0: ref, 1: torch.nn.functional.gelu(ref), 2: torch.tanh(ref)}[act]
    assert y.shape == (M, N)
    err = (y.float() - ref).abs().max().item()
    assert err < 3e-2 * max(1.0, ref.abs().max().item()), err


def test_linear_partial_tile_leaves_neighbours():
    # the store predicate: nothing is written past column N of any row (C rows are exactly N wide)
    M, N, K = 8192, 384, 768
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    ys = [native.lib().linear(x, w, None, 0, None) for _ in range(2)]
    assert torch.equal(ys[0], ys[1])
    torch.testing.assert_close(ys[0].float(), (x.float() @ w.float().t()), rtol=2e-2, atol=0.5)
