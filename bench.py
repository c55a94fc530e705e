"""Headline benchmark: training impressions/s of the federated news recommender.

BASELINE.json metric: "impressions/sec/node per FedAvg round + MIND AUC, 8 client-GPUs";
config 2: Gradient_Averaging with 1 GPU = 1 client, DistilBERT text encoder (frozen,
random init -- no pretrained weights offline) + 20-head user encoder, bf16 backbone.

One timed *step* = one synchronous federated gradient-averaging step on every client:
sample a batch of ``--batch`` impressions from the client's private synthetic MIND shard
(1 positive + 4 negatives, 50-item history) -> de-duplicate the batch's news -> full
6-layer DistilBERT forward over the unique titles (hand-written MFMA kernels) ->
text head -> user encoder -> sigmoid-CE loss -> backward (user encoder, per-news
gradient segment sum, text-head VJP) -> RCCL all-reduce of the 1.16M trainable grads ->
fused Adam.  Nothing is cached across steps (no news-vector or hidden-state cache).  The
next batch's sampling + dedup run on a lookahead stream during the current step, and (N > 1)
the all-reduce + Adam on a side stream during the next step's frozen-backbone forward.

``value`` = total impressions/s over all GPUs (weak scaling: ``--batch`` per GPU).
``vs_baseline`` divides by the reference's best measured throughput, 1.87 impressions/s
(CPU, bs 16).  After timing, an untimed validation pass reports the
AUC on the client's validation split (random-init model after W+K steps).

Single GPU: ``python bench.py``; N GPUs: ``torchrun --nproc-per-node N bench.py --gpus N``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

REF_IMPRESSIONS_PER_S = 1.87  # BASELINE.md §2 (reference code, bs 16)
METRIC = "impressions/sec/node per FedAvg round + MIND AUC, 8 client-GPUs"
_DB = "DistilBERT-base text encoder (6L/768/12H, frozen, random init) + additive head + 20-head user encoder"
MODELS = {2: _DB, 3: _DB, 4: _DB,
          5: "BERT-base-shaped text encoder (12L/768/12H, UNFROZEN, random init) + additive head + 20-head user encoder"}
MODES = {2: "Gradient_Averaging (RCCL all-reduce of flat 4.66 MB grad bucket per step)",
         3: "Parameter_Averaging (local Adam steps, RCCL all-reduce of the parameters every {k} steps)",
         4: "Gradient_Averaging + LDP (fused per-occurrence clip C=2 + Gaussian noise, eps=10 calibrated)",
         5: "Gradient_Averaging with secure aggregation (pairwise-masked int32 RCCL all-reduce of all 110M grads)"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="impressions per GPU per step")
    ap.add_argument("--preset", default="mind-small")
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5],
                    help="BASELINE.json config: 2 GA (headline), 3 parameter averaging every --pa-every "
                         "steps, 4 GA + fused LDP, 5 unfrozen BERT-base + secure-aggregation GA")
    ap.add_argument("--pa-every", type=int, default=8)
    ap.add_argument("--dp-epsilon", type=float, default=10.0)
    ap.add_argument("--valid-limit", type=int, default=2048)
    ap.add_argument("--no-valid", action="store_true")
    ap.add_argument("--profile-phases", action="store_true")
    ap.add_argument("--backbone", default="", help="test-only override of the backbone preset (e.g. 'tiny' for the "
                                                    "multi-process CPU test); the reported model says so")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    from fedrec_with_pytorchdistributed_amd.config import FedRecConfig
    from fedrec_with_pytorchdistributed_amd.data.synthetic import SynthSpec, SyntheticCorpus
    from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
    from fedrec_with_pytorchdistributed_amd.ops import native
    from fedrec_with_pytorchdistributed_amd.parallel import dist as fdist
    from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine

    ctx = fdist.init("client", "auto", timeout_s=900)
    world = ctx.world
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = ctx.device
    if dev.type == "cuda":
        native.lib()  # hard requirement on the GPU path

    from fedrec_with_pytorchdistributed_amd.config import BackboneConfig
    from fedrec_with_pytorchdistributed_amd.parallel import comm
    from fedrec_with_pytorchdistributed_amd.privacy.rdp import calibrate_client_sigma

    cfg = FedRecConfig(mode="grad_avg" if args.config != 3 else "param_avg", batch_size=args.batch, seed=0)
    if args.config == 3:
        cfg.local_update = "per_step"
    if args.config == 5:
        cfg.backbone = BackboneConfig.preset("bert-base")  # 12 layers, unfrozen
    model_name = MODELS[args.config]
    if args.backbone:
        frozen = cfg.backbone.frozen
        cfg.backbone = BackboneConfig.preset(args.backbone)
        cfg.backbone.frozen = frozen
        model_name = f"TEST ONLY: {args.backbone} backbone (not the BASELINE model)"
    torch.manual_seed(0)  # same init on every client (GA keeps them identical)
    model = FedRecModel(cfg).to(dev)
    model.build_flat()
    spec = SynthSpec.preset(args.preset)
    corpus = SyntheticCorpus(spec)
    shard = corpus.client_shard(ctx.rank, world)
    if args.config == 5:
        ar = fdist.make_secure_grad_allreduce(ctx)
    elif args.config == 3:
        ar = None
    else:
        ar = fdist.make_grad_allreduce(ctx)
    eng = LocalEngine(cfg, model, shard, dev, rank=ctx.rank, grad_allreduce=ar)
    if args.config == 4:
        cfg.dp.enabled, cfg.dp.epsilon = True, args.dp_epsilon
        eng.sigma = calibrate_client_sigma(cfg.dp.epsilon, cfg.dp.delta, cfg.batch_size, len(shard.train), cfg.dp.epochs)
    pa_state = {"n": 0}

    def step(pre):
        loss = eng.train_prepared(pre)
        if args.config == 3:
            pa_state["n"] += 1
            if world > 1 and pa_state["n"] % args.pa_every == 0:
                comm.allreduce_(model.sync_tensors(False), ctx.data_group, scale=1.0 / world)
        return loss

    # batches: sampled on the device inside the timed loop, one step ahead -- the next batch's
    # sampling + dedup run on the engine's lookahead stream while the current step computes
    it = iter(())
    epoch = [0]

    def next_batch():
        nonlocal it
        while True:
            pre = eng._next_prepared(it)
            if pre is not None:
                return pre
            it = iter(eng.sampler.epoch(epoch[0]))
            epoch[0] += 1

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    pre = next_batch()
    for _ in range(args.warmup):
        step(pre)
        pre = next_batch()
    sync()
    if ctx.initialized:
        dist.barrier(group=ctx.ctrl_group)
    sync()
    t0 = time.perf_counter()
    losses = []
    uniq = []  # unique titles per step (the backbone's work; it varies by batch and client)
    for _ in range(args.steps):
        if pre.dedup is not None:
            uniq.append(int(pre.dedup[0].numel()))
        losses.append(step(pre))
        pre = next_batch()  # the batch of the step after this one (K prepares per K steps)
    sync()
    if ctx.initialized:
        dist.barrier(group=ctx.ctrl_group)
    sync()
    elapsed = time.perf_counter() - t0
    fastest = elapsed
    u_mean = float(np.mean(uniq)) if uniq else None
    if ctx.initialized:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctx.ctrl_group)
        tmin = torch.tensor([fastest], dtype=torch.float64)
        dist.all_reduce(tmin, op=dist.ReduceOp.MIN, group=ctx.ctrl_group)
        elapsed, fastest = float(t.item()), float(tmin.item())
        if u_mean is not None:
            tu = torch.tensor([u_mean], dtype=torch.float64)
            dist.all_reduce(tu, group=ctx.ctrl_group)
            u_mean = float(tu.item()) / world
    loss = float(torch.stack(losses).float().mean())
    if ctx.initialized:  # FEDREC_COLL_CHECK=1: every client issued the same collective sequence
        from fedrec_with_pytorchdistributed_amd.parallel.collcheck import CHECK
        CHECK.verify(ctx.ctrl_group, "bench")

    # untimed: the data-plane share of a step -- the same flat-bucket RCCL all-reduce the GA
    # step issues, alone, averaged over 20 calls (bus bandwidth = 2 (W-1)/W x bytes / time)
    comm_ms = busbw = None
    if ctx.initialized and world > 1 and dev.type == "cuda" and args.config in (2, 4):
        g = torch.zeros_like(model.flat.grad)
        for _ in range(3):
            dist.all_reduce(g, group=ctx.data_group)
        sync()
        dist.barrier(group=ctx.ctrl_group)
        t1 = time.perf_counter()
        for _ in range(20):
            dist.all_reduce(g, group=ctx.data_group)
        sync()
        ct = torch.tensor([(time.perf_counter() - t1) / 20], dtype=torch.float64)
        dist.all_reduce(ct, op=dist.ReduceOp.MAX, group=ctx.ctrl_group)
        comm_ms = 1000.0 * float(ct.item())
        busbw = 2.0 * (world - 1) / world * g.numel() * g.element_size() / (comm_ms / 1000.0) / 1e9

    auc = None
    if not args.no_valid:
        m = eng.validate(batch_size=256, limit=args.valid_limit)
        vals = np.array([m["valid_auc"] * m["n_valid"], m["n_valid"]], dtype=np.float64)
        if ctx.initialized:
            tv = torch.tensor(vals)
            dist.all_reduce(tv, group=ctx.ctrl_group)
            vals = tv.numpy()
        auc = float(vals[0] / max(vals[1], 1))

    imps = args.batch * args.steps * world
    value = imps / elapsed
    if ctx.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "impressions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / REF_IMPRESSIONS_PER_S, 2),
            "dtype": "bf16" if dev.type == "cuda" else "fp32",
            "data": f"synthetic ({args.preset} MIND-format shard per client, random-init weights)",
            "config": {
                "model": model_name,
                "global_batch": args.batch * world,
                "seq_len": cfg.title_len,
                "history_len": cfg.max_his_len,
                "parallelism": f"dp{world}",
                "mode": MODES[args.config].format(k=args.pa_every),
                "baseline_config": args.config,
            },
            "train_loss": round(loss, 5),
            "fastest_rank_ms_per_step": round(1000.0 * fastest / args.steps, 3),
            "unique_titles_per_step": None if u_mean is None else round(u_mean, 1),
            "grad_allreduce_ms": None if comm_ms is None else round(comm_ms, 4),
            "grad_allreduce_busbw_GBps": None if busbw is None else round(busbw, 2),
            "valid_auc": None if auc is None else round(auc, 4),
        }
        print(json.dumps(out), flush=True)
    fdist.shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
