"""HIP-graph replay of the per-step forward + backward (cached config-2 step) equals the
eager step: same losses, same parameters after several Adam steps, across unique-title
buckets (padded unique lists) and a batch-shape change."""
import copy

import pytest
import torch

from fedrec_with_pytorchdistributed_amd.config import BackboneConfig, FedRecConfig
from fedrec_with_pytorchdistributed_amd.data.synthetic import make_client_shards
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine

pytestmark = pytest.mark.gpu


def _engines(dev, batch=16):
    cfg = FedRecConfig(mode="grad_avg", batch_size=batch, user_dropout=0.0)
    cfg.backbone = BackboneConfig(name="distilbert-2l", n_layers=2)
    torch.manual_seed(0)
    m0 = FedRecModel(cfg).to(dev)
    m1 = copy.deepcopy(m0)
    m0.build_flat()
    m1.build_flat()
    shard = make_client_shards("small", 1)[0]
    c0 = copy.deepcopy(cfg)
    c0.step_graph = "off"
    c1 = copy.deepcopy(cfg)
    c1.step_graph = "on"
    return LocalEngine(c0, m0, shard, dev), LocalEngine(c1, m1, shard, dev)


def test_graph_step_matches_eager(dev):
    e0, e1 = _engines(dev)
    assert e1.step_graphs and not e0.step_graphs
    batches = [b for _, b in zip(range(6), e0.sampler.epoch(0))]
    # a smaller last batch: a second batch shape, a second graph
    small = tuple(t[:5] for t in batches[-1])
    batches.append(small)
    # the device sampler ran on the current stream; prepare() dedups on the lookahead stream,
    # which must not read the batches before they exist
    torch.cuda.synchronize()
    l0, l1 = [], []
    for cand, his in batches:
        p0 = e0.prepare(lambda: (cand, his))
        p1 = e1.prepare(lambda: (cand, his))
        l0.append(float(e0.train_prepared(p0)))
        l1.append(float(e1.train_prepared(p1)))
    torch.cuda.synchronize()
    assert len(e1._graphs) >= 2  # several (shape, bucket) graphs were captured and replayed
    for a, b in zip(l0, l1):
        assert abs(a - b) < 1e-4, (l0, l1)
    p0, p1 = e0.model.flat.flat, e1.model.flat.flat
    rel = float((p1 - p0).norm() / p0.norm())
    # seven Adam steps over gradients that differ in fp32 summation order (the graph pads the
    # unique-title list: other split-K partitions); Adam's normalisation carries that to ~1e-5,
    # and the bf16 rounding of the user side's dQ|dK|dV (a GEMM operand, rounded once by its
    # producer) turns some of those last-bit differences into bf16-ulp ones in the Q|K|V bias
    # gradients: 2.5e-5 measured
    assert rel < 5e-5, rel
    # one client: Adam ran inside the replayed graphs with its step count on the device
    assert any(k[-2] for k in e1._graphs), "the step graphs should carry the optimizer (no all-reduce)"
    assert e1.model.flat.step == e0.model.flat.step == len(batches)
    assert int(e1._adam_step_dev.item()) == e1.model.flat.step
    # an eager step in between (e.g. a graph-cache miss) keeps the device count in step
    cand, his = batches[0]
    for e in (e0, e1):
        e.train_step(*(t for t in e.prepare(lambda: (cand, his))[:2]))
    p2 = e1.prepare(lambda: (cand, his))
    q2 = e0.prepare(lambda: (cand, his))
    assert abs(float(e0.train_prepared(q2)) - float(e1.train_prepared(p2))) < 1e-4
    torch.cuda.synchronize()
    assert int(e1._adam_step_dev.item()) == e1.model.flat.step == e0.model.flat.step
    rel = float((e1.model.flat.flat - e0.model.flat.flat).norm() / e0.model.flat.flat.norm())
    assert rel < 5e-5, rel  # two more Adam steps of bf16-rounding differences
    # the replayed graph wrote the gradient of the LAST step into the same flat buffer (the
    # in-graph Adam gathers it from the step's gradient tensors: no separate copy launch)
    g0, g1 = e0.model.flat.grad, e1.model.flat.grad
    assert float((g1 - g0).norm()) <= 2e-2 * float(g0.norm()) + 1e-8


def test_graph_with_ldp_noise_draws_fresh_noise(dev):
    """LDP under the captured step: the fused user step's noise offset is the device step
    counter, so every replay draws fresh noise (the host offset would be frozen in the graph).
    Two replays of the same batch give different gradients, and a graph step equals the eager
    step at the same counter value (same Philox draws)."""
    cfg = FedRecConfig(mode="grad_avg", batch_size=8)
    cfg.backbone = BackboneConfig(name="distilbert-2l", n_layers=2)
    cfg.dp.enabled = True
    shard = make_client_shards("tiny", 1)[0]
    engines = []
    for graphs in ("on", "off"):
        torch.manual_seed(0)
        c = copy.deepcopy(cfg)
        c.step_graph = graphs
        m = FedRecModel(c).to(dev)
        m.build_flat()
        e = LocalEngine(c, m, shard, dev)
        e.sigma = 1.0
        e.build_cache()
        engines.append(e)
    eg, ee = engines
    assert eg.step_graphs and eg.fused_user
    cand, his = next(iter(eg.sampler.epoch(0)))
    torch.cuda.synchronize()
    pre = eg.prepare(lambda: (cand, his))
    lg = eg._graph_step(pre)
    assert lg is not None and len(eg._graphs) == 1
    g1 = eg.model.flat.grad.clone()
    eg._graph_step(pre)  # same batch, next counter value: fresh noise
    g2 = eg.model.flat.grad.clone()
    assert float((g1 - g2).norm()) > 1e-6 * float(g1.norm())
    # eager step at the same counter as the second replay: same noise, same gradient
    pre2 = ee.prepare(lambda: (cand, his))
    ee._rng_step.fill_(int(eg._rng_step.item()) - 1)
    ee.forward_backward(pre2.cand, pre2.his, pre2)
    ge = ee.model.flat.grad
    assert float((ge - g2).norm()) <= 2e-2 * float(g2.norm()) + 1e-8
