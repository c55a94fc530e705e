"""Headline benchmark: training impressions/s of the federated news recommender.

BASELINE.json metric: "impressions/sec/node per FedAvg round + MIND AUC, 8 client-GPUs";
config 2: Gradient_Averaging with 1 GPU = 1 client, DistilBERT text encoder (frozen,
random init -- no pretrained weights offline) + 20-head user encoder, bf16 backbone.

Before anything is timed, every client encodes all titles of its shard once with the
frozen 6-layer DistilBERT (hand-written MFMA kernels) into an HBM-resident hidden-state
cache ``[N, 50, 768]`` bf16 (``--news-cache none`` = the round-1 path that
re-encodes the batch's unique titles every step).  The build is timed on its own
(``cache_build_ms``), after an untimed pass of ``--cache-warm`` titles (512) through the
same backbone -- the warm-up steps' counterpart: the kernels' first launches in a process
(~25 ms) are not part of the build's work.

One timed *step* = one synchronous federated gradient-averaging step on every client:
sample a batch of ``--batch`` impressions from the client's private synthetic MIND shard
(1 positive + 4 negatives, 50-item history) -> de-duplicate the batch's news -> gather the
unique titles' cached hidden states -> trainable text head (additive attention + FC 400)
-> user encoder -> sigmoid-CE loss -> backward (user encoder, per-news gradient segment
sum, text-head VJP) -> RCCL all-reduce of the 1.16M trainable grads -> fused Adam.  The
next batch's sampling + dedup run on a lookahead stream during the current step.

``value`` = total impressions/s over all GPUs (weak scaling: ``--batch`` per GPU) with the
cache build CHARGED to the timed steps: ``ms_per_step = (timed K steps + build x K /
steps_per_epoch) / K`` -- the build is amortised over one local epoch only, although the
cache of a frozen backbone stays valid for the whole run.  ``steady_ms_per_step`` is the
timed window alone.  ``vs_baseline`` divides by the reference's best measured throughput,
1.87 impressions/s (CPU fp32, bs 16): a like-for-like speedup it is not.

After the timed window (``--round``, default on for the cached configs) one full FedAvg
round is timed end to end: a whole local epoch of GA steps over the client's shard, the
validation pass over its whole validation split, and the closing metrics all-reduce;
``round_s`` / ``round_impressions_per_s`` report it and ``valid_auc`` comes from it.

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
MODES = {2: "Gradient_Averaging (all-reduce of the flat 4.66 MB grad bucket per step: {ar})",
         3: "Parameter_Averaging (local Adam steps, RCCL all-reduce of the parameters every {k} steps)",
         4: "Gradient_Averaging + LDP (fused per-occurrence clip C=2 + Gaussian noise, eps=10 calibrated; "
            "grad all-reduce: {ar})",
         5: "Gradient_Averaging with secure aggregation (pairwise-masked int32 RCCL all-reduce of all 110M grads "
            "in 28 MB buckets during the backward)"}


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
    ap.add_argument("--cache-warm", type=int, default=512,
                    help="titles run through the backbone (result dropped) before the timed cache build")
    ap.add_argument("--profile-phases", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the untimed learning probe after the round")
    ap.add_argument("--step-events", action="store_true",
                    help="diagnostic: a timing event after every timed step's launch (device interval per step)")
    ap.add_argument("--news-cache", default="auto", choices=["auto", "hidden", "none"],
                    help="HBM hidden-state cache of the frozen backbone (none = re-encode every step)")
    ap.add_argument("--round", default="auto", choices=["auto", "on", "off"],
                    help="time one full FedAvg round (local epoch + validation) after the timed steps")
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
    # N > 1: exact all-reduce self-check of the data group (RCCL on the node) before anything is
    # timed; a wrong sum raises here and the run exits non-zero
    selfcheck = fdist.selfcheck(ctx, log=lambda m: print(m, file=sys.stderr, flush=True))

    from fedrec_with_pytorchdistributed_amd.config import BackboneConfig
    from fedrec_with_pytorchdistributed_amd.parallel import comm
    from fedrec_with_pytorchdistributed_amd.privacy.rdp import calibrate_client_sigma

    cfg = FedRecConfig(mode="grad_avg" if args.config != 3 else "param_avg", batch_size=args.batch, seed=0)
    cfg.news_cache = args.news_cache
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
        ar = None  # bucketed masked all-reduce during the backward (engine.set_reducer below)
    elif args.config == 3:
        ar = None
    else:
        # N > 1: "auto" = the device-epoch IPC all-reduce inside the step graph when it checks
        # out against RCCL on this node (and is not slower in isolation), else RCCL, eager
        ar = fdist.make_grad_allreduce(ctx, choice=os.environ.get("FEDREC_ALLREDUCE", "auto"),
                                       log=lambda m: print(m, file=sys.stderr, flush=True),
                                       nelem=model.flat.grad.numel())
    eng = LocalEngine(cfg, model, shard, dev, rank=ctx.rank, grad_allreduce=ar)
    if args.config == 5:
        eng.set_reducer(fdist.make_bucket_reducer(ctx, model.flat, secure=True))
    if args.config == 4:
        cfg.dp.enabled, cfg.dp.epsilon = True, args.dp_epsilon
        eng.sigma = calibrate_client_sigma(cfg.dp.epsilon, cfg.dp.delta, cfg.batch_size, len(shard.train), cfg.dp.epochs)
    # N > 1: the clients build the hidden-state cache cooperatively -- each encodes 1/W of the
    # public catalog and the shares are all-gathered over the data plane (parallel/catalog.py);
    # the plan's id exchange is charged with the build
    from fedrec_with_pytorchdistributed_amd.parallel import catalog

    plan = catalog.attach(eng, ctx)
    pa_state = {"n": 0}
    pa_ipc = fdist.data_ipc(ctx) if (args.config == 3 and dev.type == "cuda") else None

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def max_over_ranks(x: float, op=None) -> float:
        if not ctx.initialized:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=op or dist.ReduceOp.MAX, group=ctx.ctrl_group)
        return float(t.item())

    # the HBM hidden-state cache, built once before warm-up and timed on its own (every
    # client builds its own in parallel; the slowest one counts)
    if eng.hcache is not None and args.cache_warm > 0:  # untimed, like the warm-up steps
        eng.hcache.warm(args.cache_warm)
    cache_s = eng.build_cache()
    cache_info = None
    if cache_s is not None:
        cache_info = {k: (round(1000.0 * v, 2) if k.endswith("_s") else v) for k, v in eng.hcache.build_info.items()}
        cache_info = {(k[:-2] + "_ms") if k.endswith("_s") else k: v for k, v in cache_info.items()}
        if plan is not None:
            cache_s += plan.plan_s  # one-off per run, charged like the build
        cache_s = max_over_ranks(cache_s)
    steps_per_epoch = -(-len(shard.train) // args.batch)
    steps_per_epoch = int(max_over_ranks(steps_per_epoch, dist.ReduceOp.MIN if ctx.initialized else None))

    def step(pre):
        loss = eng.train_prepared(pre)
        if args.config == 3:
            pa_state["n"] += 1
            if world > 1 and pa_state["n"] % args.pa_every == 0:
                comm.allreduce_(model.sync_tensors(False), ctx.data_group, scale=1.0 / world, ipc=pa_ipc)
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
    host_step = host_next = 0.0  # host time spent launching steps / preparing batches (diagnostic)
    wait0 = eng.host_wait_s  # ... of which blocked on the run-ahead bound (waiting for the device)
    counts0 = dict(eng.counts)
    # --step-events (diagnostic, off by default): a timing event after every step's launch
    # on the main stream -- where the device time of the timed window goes (start-up, per step, tail)
    evs = [] if (args.step_events and dev.type == "cuda") else None
    if evs is not None:
        evs.append(torch.cuda.Event(enable_timing=True))
        evs[-1].record()
    for _ in range(args.steps):
        if pre.dedup is not None:
            uniq.append(int(pre.dedup[0].numel()))
        h0 = time.perf_counter()
        losses.append(step(pre))
        h1 = time.perf_counter()
        if evs is not None:
            evs.append(torch.cuda.Event(enable_timing=True))
            evs[-1].record()
        pre = next_batch()  # the batch of the step after this one (K prepares per K steps)
        host_step += h1 - h0
        host_next += time.perf_counter() - h1
    waited = eng.host_wait_s - wait0  # read now: the round below adds its own waits
    timed_kinds = {k: v - counts0.get(k, 0) for k, v in eng.counts.items()}  # graph replays / captures / eager
    sync()
    if ctx.initialized:
        dist.barrier(group=ctx.ctrl_group)
    sync()
    elapsed = time.perf_counter() - t0
    fastest = elapsed
    if evs is not None:
        iv = [evs[i].elapsed_time(evs[i + 1]) for i in range(len(evs) - 1)]
        print(json.dumps({"bench_events_ms": {"wall": round(1000.0 * elapsed, 4),
                                               "device_first_to_last": round(evs[0].elapsed_time(evs[-1]), 4),
                                               "per_step": [round(x, 4) for x in iv]}}), file=sys.stderr, flush=True)
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

    # untimed: the data-plane share of a step -- the bucket the step all-reduces, alone, RCCL
    # vs the custom IPC all-reduce (bus bandwidth = 2 (W-1)/W x bytes / time): configs 2-4 the
    # flat fp32 4.66 MB bucket, config 5 one 28 MB int32 (masked) bucket of the reducer
    comm_ms = busbw = ipc_info = None
    if ctx.initialized and world > 1 and dev.type == "cuda":
        if args.config == 5:
            g = torch.zeros(7 << 20, dtype=torch.int32, device=dev)
        else:
            g = torch.zeros_like(model.flat.grad)
        nbytes = g.numel() * g.element_size()

        def timed(fn, reps=20):
            for _ in range(3):
                fn(g)
            sync()
            dist.barrier(group=ctx.ctrl_group)
            t1 = time.perf_counter()
            for _ in range(reps):
                fn(g)
            sync()
            ct = torch.tensor([(time.perf_counter() - t1) / reps], dtype=torch.float64)
            dist.all_reduce(ct, op=dist.ReduceOp.MAX, group=ctx.ctrl_group)
            return 1000.0 * float(ct.item())

        comm_ms = timed(lambda x: dist.all_reduce(x, group=ctx.data_group))
        busbw = 2.0 * (world - 1) / world * nbytes / (comm_ms / 1000.0) / 1e9
        # the custom IPC all-reduce (one-shot / two-shot over xGMI) on the same bucket; its result
        # is checked against RCCL's first.  A failure is reported, not fatal.
        try:
            ipc = fdist.make_ipc_allreduce(ctx)
            if g.dtype == torch.int32:
                a = torch.randint(-2**30, 2**30, g.shape, dtype=torch.int32, device=dev)
            else:
                a = torch.randn_like(g)
            b = a.clone()
            dist.all_reduce(a, group=ctx.data_group)
            ipc.allreduce_(b)
            sync()
            ok = bool(torch.equal(a, b)) if g.dtype == torch.int32 else bool(torch.allclose(a, b, rtol=1e-5, atol=1e-6))
            ipc_ms = timed(ipc.allreduce_)
            ipc_info = {"bucket_MB": round(nbytes / 2**20, 2), "dtype": str(g.dtype).split(".")[-1],
                        "ms": round(ipc_ms, 4), "matches_rccl": ok, "status": ipc.status(),
                        "busbw_GBps": round(2.0 * (world - 1) / world * nbytes / (ipc_ms / 1000.0) / 1e9, 2)}
            ipc.close()
        except Exception as e:  # pragma: no cover - depends on the node
            ipc_info = {"error": repr(e)[:300]}

    def reduce_valid(m):
        vals = np.array([m["valid_auc"] * m["n_valid"], m["n_valid"]], dtype=np.float64)
        if ctx.initialized:
            tv = torch.tensor(vals)
            dist.all_reduce(tv, group=ctx.ctrl_group)
            vals = tv.numpy()
        return float(vals[0] / max(vals[1], 1))

    # one full FedAvg round, end to end: a whole local epoch of synchronous steps (every
    # client runs the same number of steps, so the collectives match), validation over the
    # whole validation split, the closing metrics all-reduce
    do_round = args.round == "on" or (args.round == "auto" and eng.hcache is not None)
    rnd = None
    auc = None
    if do_round:
        eng.prepare_validation(256)  # the validation split's device arrays: setup, like the cache
        eng.sync_params()
        sync()
        if ctx.initialized:
            dist.barrier(group=ctx.ctrl_group)
        t1 = time.perf_counter()
        hook = None
        if args.config == 3 and world > 1:
            hook = (lambda n: comm.allreduce_(model.sync_tensors(False), ctx.data_group, scale=1.0 / world,
                                              ipc=pa_ipc)
                    if n % args.pa_every == 0 else None)
        st = eng.train_epoch(max_steps=steps_per_epoch, step_hook=hook)
        t2 = time.perf_counter()
        mv = eng.validate(batch_size=256)
        auc = reduce_valid(mv)
        sync()
        if ctx.initialized:
            dist.barrier(group=ctx.ctrl_group)
        t3 = time.perf_counter()
        round_s = max_over_ranks(t3 - t1)
        rnd = {"round_s": round(round_s, 4), "round_train_s": round(max_over_ranks(t2 - t1), 4),
               "round_valid_s": round(max_over_ranks(t3 - t2), 4), "round_steps": st["steps"],
               "round_impressions_per_s": round(st["steps"] * args.batch * world / round_s, 2),
               "round_train_loss": round(st["training_loss"], 5), "round_valid_impressions": int(mv["n_valid"])}
        if cache_s is not None:  # a first round also pays for the cache build
            rnd["first_round_s"] = round(round_s + cache_s, 4)
    elif not args.no_valid:
        auc = reduce_valid(eng.validate(batch_size=256, limit=args.valid_limit))

    # learning probe (after everything above, untimed): the reference's sigmoid-CE scorer keeps
    # this shard at chance (docs/PARITY.md: the reference's own loop does too), so the round's
    # valid_auc says nothing about whether the engine learns at the headline shape.  One more
    # local epoch with the plain-CE scorer (score_act=identity, the quality runs' setting) from
    # where the round left the model, then the validation AUC.  The step graphs were captured
    # with the reference scorer: they are dropped and re-captured.
    probe = None
    if do_round and not args.no_probe:
        cfg.score_act = "identity"
        eng._graphs.clear()
        eng.sync_params()
        sync()
        if ctx.initialized:
            dist.barrier(group=ctx.ctrl_group)
        tp = time.perf_counter()
        stp = eng.train_epoch(max_steps=steps_per_epoch)
        mvp = eng.validate(batch_size=256)
        probe = {"score_act": "identity", "lr": cfg.lr, "epochs": 1, "steps": stp["steps"],
                 "train_loss": round(stp["training_loss"], 5), "valid_auc": round(reduce_valid(mvp), 4),
                 "wall_s": round(max_over_ranks(time.perf_counter() - tp), 3)}

    amort = 0.0 if cache_s is None else cache_s * args.steps / steps_per_epoch
    charged = elapsed + amort
    imps = args.batch * args.steps * world
    value = imps / charged
    ar_desc = "none"
    if ar is not None:
        ar_desc = ("device-epoch IPC over xGMI inside the step graph" if ar.kind == "ipc" and ar.capturable else
                   f"{ar.kind}, " + ("inside the step graph" if ar.capturable else "eager on the optimizer stream"))
    if ctx.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "impressions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * charged / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / REF_IMPRESSIONS_PER_S, 2),
            "vs_baseline_note": ("value / 1.87 imp/s: the reference code measured on an 8-core CPU in fp32 "
                                 "(BASELINE.md table 2; the reference publishes no throughput) -- a hardware + "
                                 "design ratio, not a like-for-like speedup"),
            "dtype": "bf16" if dev.type == "cuda" else "fp32",
            "data": f"synthetic ({args.preset} MIND-format shard per client, random-init weights)",
            "config": {
                "model": model_name,
                "global_batch": args.batch * world,
                "seq_len": cfg.title_len,
                "history_len": cfg.max_his_len,
                "parallelism": f"dp{world}",
                "mode": (MODES[args.config].format(k=args.pa_every, ar=ar_desc) if world > 1 else
                         MODES[args.config].split(" (")[0] + " (1 client: no all-reduce issued)"),
                "baseline_config": args.config,
            },
            "train_loss": round(loss, 5),
            "news_cache": "hidden" if eng.hcache is not None else "none",
            "cache_build_ms": None if cache_s is None else round(1000.0 * cache_s, 2),
            "cache_warm_titles": args.cache_warm if cache_s is not None else None,
            "cache_build": cache_info,  # rank 0's breakdown (cooperative at N > 1: 1/W encoded + gather)
            "steps_per_epoch": steps_per_epoch,
            "steady_ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            # launch + next_batch include the host blocking on the run-ahead bound (run_ahead_wait:
            # the device is the limit then); host_work = what the host itself spends per step
            "host_ms_per_step": {"launch": round(1000.0 * host_step / args.steps, 4),
                                 "next_batch": round(1000.0 * host_next / args.steps, 4),
                                 "run_ahead_wait": round(1000.0 * waited / args.steps, 4),
                                 "host_work": round(1000.0 * (host_step + host_next - waited)
                                                    / args.steps, 4)},
            "cache_amortized_ms_per_step": round(1000.0 * amort / args.steps, 4),
            "timed_step_kinds": timed_kinds,
            "fastest_rank_ms_per_step": round(1000.0 * fastest / args.steps, 3),
            "unique_titles_per_step": None if u_mean is None else round(u_mean, 1),
            "grad_allreduce": None if ar is None else {"kind": ar.kind, "in_step_graph": bool(ar.capturable),
                                                       "probe": getattr(ar, "probe", None),
                                                       "replays_with_optimizer": eng.counts["replays_with_optimizer"],
                                                       "eager_optimizer_steps": eng.counts["eager_optimizer_steps"]},
            "grad_allreduce_ms": None if comm_ms is None else round(comm_ms, 4),
            "grad_allreduce_busbw_GBps": None if busbw is None else round(busbw, 2),
            "valid_auc": None if auc is None else round(auc, 4),
            "data_group": None if not (ctx.initialized and ctx.data_group is not None) else
            {"backend": dist.get_backend(ctx.data_group), "size": dist.get_world_size(ctx.data_group)},
            "data_plane_selfcheck": selfcheck or None,
            "ipc_allreduce": ipc_info,
            "learning_probe": probe,
        }
        if rnd is not None:
            out.update(rnd)
        print(json.dumps(out), flush=True)
    fdist.shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
