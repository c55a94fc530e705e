"""Launch fusions of the config-2 step against their unfused forms, through the whole engine:
each switch (a module flag of ops/functional.py) only changes where the arithmetic runs, not the
arithmetic, so after a few training steps the losses, gradients and parameters are bitwise
those of the unfused launches.

* FUSED_QKV_ATTN: the user encoder's Q|K|V projection inside the attention forward launch and
  the pool's input-gradient GEMM inside the attention backward launch vs their own small-GEMM
  launches (the text head's pool backward + g rewrite fusion, pinned here until round 5, lost
  its unfused form in round 6: tests/test_text_head_gpu.py checks it against an fp32 oracle);
* DEFER_REDUCE: the text fc backward's split-K reduce in the head's reduce launch (see also
  test_deferred_reduce_gpu.py)."""
import pytest
import torch

from fedrec_with_pytorchdistributed_amd.config import FedRecConfig
from fedrec_with_pytorchdistributed_amd.data.synthetic import make_client_shards
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
from fedrec_with_pytorchdistributed_amd.ops import functional as OF
from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine

pytestmark = pytest.mark.gpu


def _run(dev, steps, mask_padding=False):
    cfg = FedRecConfig(mode="grad_avg", batch_size=32)
    cfg.mask_padding = mask_padding
    torch.manual_seed(0)
    m = FedRecModel(cfg).to(dev)
    m.build_flat()
    eng = LocalEngine(cfg, m, make_client_shards("tiny", 1)[0], dev)
    if not eng.fused_head or not eng.fused_user:
        pytest.skip("this configuration does not take the fused step")
    batches = [tuple(eng.to_device(a) for a in b) for _, b in zip(range(steps), eng.sampler.epoch(0))]
    losses = [eng.train_step(*b) for b in batches]
    torch.cuda.synchronize()
    return torch.stack([torch.as_tensor(x, device=dev).float().reshape(()) for x in losses]), eng.flat.flat.clone()


@pytest.mark.parametrize("flag", ["FUSED_QKV_ATTN", "DEFER_REDUCE"])
@pytest.mark.parametrize("mask_padding", [False, True])
def test_step_fusion_is_bitwise(dev, flag, mask_padding):
    saved = getattr(OF, flag)
    out = {}
    try:
        for on in (False, True):
            setattr(OF, flag, on)
            out[on] = _run(dev, 3, mask_padding)
    finally:
        setattr(OF, flag, saved)
    assert torch.equal(out[True][0], out[False][0]), (out[True][0], out[False][0])
    assert torch.equal(out[True][1], out[False][1])
