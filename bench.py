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
fused Adam.  Nothing is cached across steps (no news-vector or hidden-state cache).

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


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="impressions per GPU per step")
    ap.add_argument("--preset", default="mind-small")
    ap.add_argument("--mode", default="grad_avg", choices=["grad_avg"])
    ap.add_argument("--valid-limit", type=int, default=2048)
    ap.add_argument("--no-valid", action="store_true")
    ap.add_argument("--profile-phases", action="store_true")
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

    cfg = FedRecConfig(mode="grad_avg", batch_size=args.batch, seed=0)
    torch.manual_seed(0)  # same init on every client (GA keeps them identical)
    model = FedRecModel(cfg).to(dev)
    model.build_flat()
    spec = SynthSpec.preset(args.preset)
    corpus = SyntheticCorpus(spec)
    shard = corpus.client_shard(ctx.rank, world)
    eng = LocalEngine(cfg, model, shard, dev, rank=ctx.rank, grad_allreduce=fdist.make_grad_allreduce(ctx))

    # batches: sampled on the fly inside the timed loop (host sampler + H2D copy)
    it = iter(())
    epoch = [0]

    def next_batch():
        nonlocal it
        while True:
            try:
                c, h = next(it)
                return eng.to_device(c), eng.to_device(h)
            except StopIteration:
                it = iter(eng.sampler.epoch(epoch[0]))
                epoch[0] += 1

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        eng.train_step(*next_batch())
    sync()
    if ctx.initialized:
        dist.barrier(group=ctx.ctrl_group)
    sync()
    t0 = time.perf_counter()
    losses = []
    for _ in range(args.steps):
        losses.append(eng.train_step(*next_batch()))
    sync()
    if ctx.initialized:
        dist.barrier(group=ctx.ctrl_group)
    sync()
    elapsed = time.perf_counter() - t0
    if ctx.initialized:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctx.ctrl_group)
        elapsed = float(t.item())
    loss = float(torch.stack(losses).float().mean())

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
            "dtype": "bf16",
            "data": f"synthetic ({args.preset} MIND-format shard per client, random-init weights)",
            "config": {
                "model": "DistilBERT-base text encoder (6L/768/12H, frozen, random init) + additive head + "
                         "20-head user encoder",
                "global_batch": args.batch * world,
                "seq_len": cfg.title_len,
                "history_len": cfg.max_his_len,
                "parallelism": f"dp{world}",
                "mode": "Gradient_Averaging (RCCL all-reduce of flat 4.66 MB grad bucket per step)",
            },
            "train_loss": round(loss, 5),
            "valid_auc": None if auc is None else round(auc, 4),
        }
        print(json.dumps(out), flush=True)
    fdist.shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
