"""Deferred split-K reduction: the text fc backward's weight-gradient reduce runs in extra blocks
of the text head's reduce launch (ops/functional.py DEFER_REDUCE, csrc/text_head.hip
head_reduce_kernel<true>).  The same reduction arithmetic either way, so one training step's
gradients and updated parameters are bitwise those of the standalone reduce launch, and the
step's kernel trace holds no splitk_reduce_kernel of its own."""
import pytest
import torch
from torch.profiler import ProfilerActivity, profile

from fedrec_with_pytorchdistributed_amd.config import FedRecConfig
from fedrec_with_pytorchdistributed_amd.data.synthetic import make_client_shards
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
from fedrec_with_pytorchdistributed_amd.ops import functional as OF
from fedrec_with_pytorchdistributed_amd.ops import native
from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine

pytestmark = pytest.mark.gpu


def _engine(dev):
    cfg = FedRecConfig(mode="grad_avg", batch_size=32)
    torch.manual_seed(0)
    m = FedRecModel(cfg).to(dev)
    m.build_flat()
    eng = LocalEngine(cfg, m, make_client_shards("tiny", 1)[0], dev)
    if not eng.fused_head:
        pytest.skip("this configuration does not take the fused text head")
    return eng


def _names(prof):
    return [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]


@pytest.mark.parametrize("steps", [1, 3])
def test_deferred_reduce_matches_standalone(dev, steps):
    out = {}
    saved = OF.DEFER_REDUCE
    try:
        for defer in (False, True):
            OF.DEFER_REDUCE = defer
            eng = _engine(dev)
            batches = [tuple(eng.to_device(a) for a in b) for _, b in zip(range(steps), eng.sampler.epoch(0))]
            for b in batches:
                eng.train_step(*b)
            torch.cuda.synchronize()
            out[defer] = (eng.flat.grad.clone(), eng.flat.flat.clone())
    finally:
        OF.DEFER_REDUCE = saved
    assert not native.lib().small_gemm_flush_pending()  # nothing left pending after the steps
    assert torch.equal(out[True][0], out[False][0])
    assert torch.equal(out[True][1], out[False][1])


def test_deferred_reduce_rides_in_head_reduce(dev):
    saved = OF.DEFER_REDUCE
    names = {}
    try:
        for defer in (False, True):
            OF.DEFER_REDUCE = defer
            eng = _engine(dev)
            batches = [tuple(eng.to_device(a) for a in b) for _, b in zip(range(2), eng.sampler.epoch(0))]
            eng.train_step(*batches[0])
            torch.cuda.synchronize()
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                eng.train_step(*batches[1])
                torch.cuda.synchronize()
            names[defer] = _names(prof)
    finally:
        OF.DEFER_REDUCE = saved

    def count(ns, key):
        return sum(1 for n in ns if key in n)

    assert count(names[False], "splitk_reduce_kernel") >= 1
    assert count(names[True], "splitk_reduce_kernel") == count(names[False], "splitk_reduce_kernel") - 1
    assert count(names[True], "head_reduce_kernel") == count(names[False], "head_reduce_kernel")
