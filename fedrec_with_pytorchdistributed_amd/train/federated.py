"""Federation drivers: the three aggregation strategies of the reference.

``run_grad_avg``   Gradient_Averaging_main.py / main.py (C13a/b, C35): synchronous DP --
                   every step the flat gradient bucket (1.16M fp32) is all-reduced over the
                   client GPUs (RCCL/xGMI) and one fused Adam step follows.  Fixes E4/E5:
                   any number of batches per epoch, BOTH encoders synchronised.
``run_param_avg``  Parameter_Averaging_main.py (C13c, C36): local training, then the
                   parameters are averaged by all-reduce once per epoch (or every
                   ``param_avg_every`` local steps) -- local SGD / serverless FedAvg.
``run_star_*``     client.py / server.py (C06-C11): a coordinator broadcasts the global
                   model, clients train ``total_epochs`` local epochs, upload, and the
                   coordinator averages (unweighted like ``server.py:49``, or weighted by
                   sample count) -- through the fault-tolerant store control plane, with
                   quorum, timeouts, NaN-rejection and optional secure aggregation; or with
                   ``allreduce`` aggregation, the clients average among themselves over RCCL
                   and only the result goes to the coordinator.

All modes write ``snapshot.pt`` in the reference layout (rank 0 / coordinator, atomic) and
JSONL metrics with the reference's metric names.
"""
from __future__ import annotations

import math
import os
import time
from typing import Tuple, Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..config import FedRecConfig
from ..data.shard import Shard
from ..data.synthetic import SynthSpec, SyntheticCorpus
from ..models.fedrec_model import FedRecModel
from ..parallel import catalog, comm
from ..parallel import secagg
from ..parallel.collcheck import CHECK
from ..parallel.control import ControlPlane, Heartbeat
from ..parallel.dist import (DistContext, data_ipc, make_bucket_reducer, make_grad_allreduce, make_secure_grad_allreduce,
                             selfcheck)
from ..privacy.rdp import calibrate_client_sigma
from ..utils import obs
from ..utils.fault import FaultInjector
from . import checkpoint as ckpt
from .engine import LocalEngine

METRIC_KEYS = ("training_loss", "validation_loss", "valid_auc", "valid_mrr", "val_ndcg@5", "val_ndcg@10")


# ---------------------------------------------------------------------------------------
def load_client_shard(cfg: FedRecConfig, ctx: DistContext) -> Shard:
    """``data_dir`` forms: a reference ``UserData`` dir (``{client}`` is replaced by the
    client index for single-node multi-client runs), or ``synthetic:<preset>[:<seed>]``."""
    k, W = max(ctx.client_index, 0), max(ctx.num_clients, 1)
    if cfg.data_dir.startswith("synthetic:"):
        parts = cfg.data_dir.split(":")
        spec = SynthSpec.preset(parts[1])
        spec.seed = int(parts[2]) if len(parts) > 2 else cfg.seed
        shard = SyntheticCorpus(spec).client_shard(k, W)
    else:
        shard = Shard.load(cfg.data_dir.replace("{client}", str(k)))
    if cfg.quirks().resplit_shard and W > 1:
        shard = shard.split_train(k, W)  # Q11: DistributedSampler re-split (client.py:249)
    return shard


def build_model(cfg: FedRecConfig, device: torch.device) -> FedRecModel:
    torch.manual_seed(cfg.seed)  # identical init on every participant
    model = FedRecModel(cfg).to(device)
    model.build_flat()
    return model


def _metrics_writer(cfg: FedRecConfig, is_writer: bool) -> obs.MetricsWriter:
    path = cfg.metrics_path or os.path.join(os.path.dirname(os.path.abspath(cfg.snapshot_path)), "metrics.jsonl")
    return obs.MetricsWriter(path if is_writer else None, cfg.run_name, cfg.wandb_project, cfg.to_dict())


def _reduce_metrics(ctx: DistContext, train: Dict, val: Dict) -> Dict:
    """Corpus-level metrics over all clients: one packed gloo all-reduce (X8 replacement)."""
    n = float(val.get("n_valid", 0))
    v = torch.tensor([train.get("training_loss", 0.0) * train.get("steps", 0), train.get("steps", 0),
                      train.get("impressions", 0), val.get("validation_loss", 0.0) * n,
                      val.get("valid_auc", 0.0) * n, val.get("valid_mrr", 0.0) * n,
                      val.get("val_ndcg@5", 0.0) * n, val.get("val_ndcg@10", 0.0) * n, n], dtype=torch.float64)
    v = torch.nan_to_num(v)
    t = torch.tensor([train.get("epoch_s", 0.0)], dtype=torch.float64)
    if ctx.initialized and ctx.num_clients > 1:
        dist.all_reduce(v, group=ctx.ctrl_group)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctx.ctrl_group)
    steps, nv = max(v[1].item(), 1), max(v[8].item(), 1)
    return {"training_loss": v[0].item() / steps, "validation_loss": v[3].item() / nv, "valid_auc": v[4].item() / nv,
            "valid_mrr": v[5].item() / nv, "val_ndcg@5": v[6].item() / nv, "val_ndcg@10": v[7].item() / nv,
            "impressions": v[2].item(), "epoch_s": t.item(), "impressions_per_s": v[2].item() / max(t.item(), 1e-9)}


def _min_over_clients(ctx: DistContext, x: int) -> int:
    if not ctx.initialized or ctx.num_clients <= 1:
        return x
    t = torch.tensor([x], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.ctrl_group)
    return int(t.item())


def _backbone_before(model: FedRecModel, full: bool) -> Optional[torch.Tensor]:
    """Fingerprint of a FROZEN backbone about to be overwritten by a ``sync=full`` collective
    (None when no check applies)."""
    if full and model.cfg.backbone.frozen:
        return model.text_encoder.DistillBert.fingerprint()
    return None


def _backbone_synced(model: FedRecModel, full: bool, before: Optional[torch.Tensor] = None) -> None:
    """Parameters were overwritten by a collective: the backbone changed iff it was part of
    the synced set (``sync=full``, or an unfrozen backbone is trainable), and only then do
    its compute pack and the HBM hidden-state cache have to be rebuilt.  A frozen backbone
    synced with ``sync=full`` is compared against its fingerprint from before the sync: the
    reference-compat full sync (Q15) moves the 270 MB every round, but between identical
    replicas it changes nothing and must not force a re-encode of every title."""
    if not model.cfg.backbone.frozen:
        model.text_encoder.DistillBert.invalidate()
    elif full:
        if before is None:
            model.text_encoder.DistillBert.invalidate()
        else:
            model.text_encoder.DistillBert.invalidate_if_changed(before)


def _sync_initial(model: FedRecModel, ctx: DistContext, full: bool) -> None:
    """DDP-style start: every client takes client 0's parameters (X6, one bucketed call)."""
    if ctx.initialized and ctx.num_clients > 1:
        before = _backbone_before(model, full)
        comm.broadcast_(model.sync_tensors(full), src=ctx.client_ranks[0], group=ctx.data_group)
        _backbone_synced(model, full, before)


def _maybe_dp(cfg: FedRecConfig, eng: LocalEngine) -> Optional[float]:
    if not cfg.dp.enabled:
        return None
    if cfg.dp.noise_multiplier is not None:
        return float(cfg.dp.noise_multiplier)
    return calibrate_client_sigma(cfg.dp.epsilon, cfg.dp.delta, cfg.batch_size, len(eng.shard.train),
                                  cfg.dp.epochs)


def _dump_flat(model: FedRecModel, ctx: DistContext) -> None:
    """Test hook: ``FEDREC_DUMP_FLAT=<dir>`` saves each rank's final trainable parameters."""
    d = os.environ.get("FEDREC_DUMP_FLAT")
    if d:
        os.makedirs(d, exist_ok=True)
        torch.save(model.flat.flat.detach().cpu(), os.path.join(d, f"rank{ctx.rank}.pt"))


def _resume(cfg: FedRecConfig, model: FedRecModel, server: Optional["ServerStep"] = None) -> Tuple[int, Dict]:
    """(next epoch, engine counters) of ``cfg.snapshot_path`` when it exists (params, Adam
    moments and RNG states are restored into ``model`` / torch; the server step's momentum into
    ``server``)."""
    if cfg.snapshot_path and os.path.exists(cfg.snapshot_path):
        info = ckpt.load_snapshot(cfg.snapshot_path, model)
        if server is not None:
            server.load(info.get("server_opt"))
        obs.log(f"resuming from {cfg.snapshot_path}: epochs_run={info['epochs_run']} -> epoch {info['next_epoch']}")
        return info["next_epoch"], info["engine"]
    return 0, {}


class ServerStep:
    """The server-side step on an averaged model (``cfg.server_lr`` / ``cfg.server_momentum``):
    ``v = momentum * v + (avg - theta_g)``, ``theta = theta_g + lr * v`` -- FedAvgM (Hsu et al.
    2019, server momentum) with a server learning rate (Reddi et al. 2021).  At lr 1 and
    momentum 0 it is the plain mean of the reference (``server.py:46-50``,
    ``Parameter_Averaging_main.py:144-148``) and does nothing.  Computed in fp64 on the host for
    the coordinator and in fp32 on the device for parameter averaging (every PA client applies it
    to the same all-reduced mean, so the clients stay bitwise identical)."""

    def __init__(self, lr: float = 1.0, momentum: float = 0.0, opt: str = "sgd", beta2: float = 0.99,
                 tau: float = 1e-3):
        if opt not in ("sgd", "adam"):
            raise ValueError(f"server_opt={opt!r}: expected sgd | adam")
        self.lr, self.momentum, self.opt = float(lr), float(momentum), opt
        self.beta2, self.tau = float(beta2), float(tau)
        self.v: Optional[torch.Tensor] = None  # sgd: the momentum buffer; adam: the first moment
        self.s: Optional[torch.Tensor] = None  # adam: the second moment

    @classmethod
    def from_cfg(cls, cfg) -> "ServerStep":
        return cls(cfg.server_lr, cfg.server_momentum, cfg.server_opt, cfg.server_beta2, cfg.server_tau)

    @property
    def active(self) -> bool:
        return self.opt == "adam" or self.lr != 1.0 or self.momentum != 0.0

    def apply(self, theta_g: torch.Tensor, avg: torch.Tensor) -> torch.Tensor:
        """The new global model from the round's global ``theta_g`` and the clients' mean."""
        if not self.active:
            return avg
        d = avg - theta_g
        if self.opt == "adam":  # FedAdam: per-coordinate normalised server step
            self.v = ((1 - self.momentum) * d if self.v is None
                      else self.v.to(d.device).mul_(self.momentum).add_(d, alpha=1 - self.momentum))
            self.s = ((1 - self.beta2) * d * d if self.s is None
                      else self.s.to(d.device).mul_(self.beta2).addcmul_(d, d, value=1 - self.beta2))
            return theta_g + self.lr * self.v / (self.s.sqrt() + self.tau)
        self.v = d if self.v is None else self.v.to(d.device).mul_(self.momentum).add_(d)
        return theta_g + self.lr * self.v

    def state(self) -> Optional[Dict]:
        if not self.active or self.v is None:
            return None
        return {"v": self.v, **({"s": self.s} if self.s is not None else {})}

    def load(self, st: Optional[Dict]) -> None:
        if st and st.get("v") is not None:
            self.v = st["v"].clone()
        if st and st.get("s") is not None:
            self.s = st["s"].clone()


# ---------------------------------------------------------------------------------------
def run_grad_avg(cfg: FedRecConfig, ctx: DistContext) -> Dict:
    selfcheck(ctx, log=obs.log)
    shard = load_client_shard(cfg, ctx)
    model = build_model(cfg, ctx.device)
    start, est = _resume(cfg, model)
    _sync_initial(model, ctx, cfg.sync == "full")
    # large trainable sets (unfrozen backbone: ~66-110M grads) reduce in ~28 MB buckets during the
    # backward; the frozen backbone's 4.66 MB head + user encoder is one flat bucket per step
    bucketed = not cfg.backbone.frozen and cfg.bucket_reducer
    if bucketed:
        ar = None
    else:
        ar = (make_secure_grad_allreduce(ctx, timeout_s=cfg.collective_timeout_s)
              if cfg.secagg.enabled else make_grad_allreduce(ctx, cfg.collective_timeout_s))
    eng = LocalEngine(cfg, model, shard, ctx.device, rank=ctx.rank, grad_allreduce=ar)
    if bucketed:
        eng.set_reducer(make_bucket_reducer(ctx, model.flat, secure=cfg.secagg.enabled,
                                            timeout_s=cfg.collective_timeout_s))
    eng.sigma = _maybe_dp(cfg, eng)
    eng.load_state(est)
    eng.epoch = start
    catalog.attach(eng, ctx)  # cooperative hidden-state cache builds over the clients
    writer = _metrics_writer(cfg, ctx.client_index == 0)
    steps = _min_over_clients(ctx, eng.sampler.num_batches())  # every rank issues the same all-reduces
    last = {}
    for epoch in range(start, cfg.total_epochs):
        eng.ensure_cache()  # a collective point: every client rebuilds a stale cache together
        tr = eng.train_epoch(max_steps=steps)
        va = eng.validate()
        CHECK.verify(ctx.ctrl_group, f"grad_avg epoch {epoch}")
        last = _reduce_metrics(ctx, tr, va)
        last.update({"epoch": epoch, "mode": "grad_avg", "clients": ctx.num_clients})
        if ctx.client_index == 0:
            writer.write(last)
            obs.log(f"[grad_avg] epoch {epoch}: " + ", ".join(f"{k}={last[k]:.4f}" for k in METRIC_KEYS))
            if cfg.save_every and (epoch % cfg.save_every == 0 or epoch == cfg.total_epochs - 1):
                ckpt.save_snapshot(cfg.snapshot_path, model, epoch, config=cfg.to_dict(), engine=eng.state())
    _dump_flat(model, ctx)
    return last


def run_param_avg(cfg: FedRecConfig, ctx: DistContext) -> Dict:
    selfcheck(ctx, log=obs.log)
    shard = load_client_shard(cfg, ctx)
    model = build_model(cfg, ctx.device)
    server = ServerStep.from_cfg(cfg)
    start, est = _resume(cfg, model, server)
    full = cfg.sync == "full"
    _sync_initial(model, ctx, full)
    eng = LocalEngine(cfg, model, shard, ctx.device, rank=ctx.rank, grad_allreduce=None)
    # the model at the last average (the server step's theta_g): every client holds the same one
    anchor = model.flat.flat.detach().clone() if server.active else None
    eng.sigma = _maybe_dp(cfg, eng)
    eng.load_state(est)
    eng.epoch = start
    catalog.attach(eng, ctx)
    writer = _metrics_writer(cfg, ctx.client_index == 0)
    W = ctx.num_clients
    sched = cfg.resolved_local_update()
    K = cfg.param_avg_every if sched == "per_step" else 0
    steps = _min_over_clients(ctx, eng.sampler.num_batches()) if K else None

    ipc = data_ipc(ctx, cfg.collective_timeout_s) if ctx.device.type == "cuda" else None

    def average():
        if ctx.initialized and W > 1:
            before = _backbone_before(model, full)
            ts = model.sync_tensors(full)
            if cfg.pa_average_moments:  # the clients' Adam moments averaged with the parameters
                ts = ts + [model.flat.m, model.flat.v]
            with obs.range("param_allreduce"):
                comm.allreduce_(ts, ctx.data_group, scale=1.0 / W, ipc=ipc)
            if anchor is not None:  # server step on the mean (same inputs on every client)
                with torch.no_grad():
                    model.flat.flat.copy_(server.apply(anchor, model.flat.flat))
                    anchor.copy_(model.flat.flat)
            _backbone_synced(model, full, before)

    hook = (lambda n: average() if n % K == 0 else None) if K else None
    last = {}
    for epoch in range(start, cfg.total_epochs):
        eng.ensure_cache()
        tr = eng.train_epoch(max_steps=steps, step_hook=hook)
        if not K or (steps or 0) % K:
            average()  # once per epoch (Parameter_Averaging_main.py:144-148)
        if ipc is not None:
            ipc.check()  # a timed-out IPC all-reduce poisoned its bucket: fail loudly
        va = eng.validate()
        CHECK.verify(ctx.ctrl_group, f"param_avg epoch {epoch}")
        last = _reduce_metrics(ctx, tr, va)
        last.update({"epoch": epoch, "mode": "param_avg", "clients": W})
        if ctx.client_index == 0:
            writer.write(last)
            obs.log(f"[param_avg] epoch {epoch}: " + ", ".join(f"{k}={last[k]:.4f}" for k in METRIC_KEYS))
            if cfg.save_every and (epoch % cfg.save_every == 0 or epoch == cfg.total_epochs - 1):
                ckpt.save_snapshot(cfg.snapshot_path, model, epoch, config=cfg.to_dict(), engine=eng.state(),
                                   server_opt=server.state())
    _dump_flat(model, ctx)
    return last


# ---------------------------------------------------------------------------------------
# star topology: coordinator + clients over the store control plane
# ---------------------------------------------------------------------------------------
def _aggregation(cfg: FedRecConfig, ctx: DistContext) -> str:
    if cfg.quorum < 1.0 or cfg.secagg.enabled or not ctx.initialized:
        return "upload"
    return os.environ.get("FEDREC_STAR_AGG", "allreduce")


def _artifact_dir(cfg: FedRecConfig) -> str:
    return os.path.dirname(os.path.abspath(cfg.snapshot_path or "snapshot.pt"))


def _client_upload_tensor(model: FedRecModel, cfg: FedRecConfig) -> torch.Tensor:
    return model.flat.flat.detach().float()


def run_star_client(cfg: FedRecConfig, ctx: DistContext, run_id: str = "star") -> Dict:
    cp = ControlPlane.from_default(run_id, cfg.round_timeout_s)
    k = ctx.client_index
    shard = load_client_shard(cfg, ctx)
    model = build_model(cfg, ctx.device)  # created ONCE: Adam moments persist across rounds
    eng = LocalEngine(cfg, model, shard, ctx.device, rank=ctx.rank, grad_allreduce=None)
    fault = FaultInjector("client", k)
    agg = _aggregation(cfg, ctx)
    full = cfg.sync == "full"
    writer = _metrics_writer(cfg, False)
    # secure aggregation: pairwise seeds by Diffie-Hellman over the control plane
    seeds_row = secure = None
    if cfg.secagg.enabled:
        kp = secagg.KeyPair()
        cp.set(f"pk/{k}", secagg.public_bytes(kp))
        pubs = [cp.get(f"pk/{j}") for j in range(ctx.num_clients)]
        seeds_row = secagg.seeds_from_publics(kp, k, pubs)
        secure = secagg.StarSecureUpload(cp, k, ctx.num_clients, seeds_row)
    r = int(cp.get("start").decode())  # the coordinator may be resuming at a later round
    # the client's own snapshot (client.py:125-127 auto-loads snapshot.pt): Adam moments + step,
    # RNG states and engine counters; the trainable parameters are overwritten by the round's
    # global model below, exactly as the reference's broadcast overwrites them
    csnap = ckpt.client_snapshot_path(cfg.snapshot_path, k) if cfg.snapshot_path else ""
    if csnap and cfg.save_every and cfg.save_every > 1:
        obs.log(f"[client {k}] save_every={cfg.save_every} does not apply to client snapshots: they are written "
                "every round (a resume from an older round would redraw LDP noise / dropout already uploaded)")
    if csnap and os.path.exists(csnap):
        info = ckpt.load_client_state(csnap, model)
        eng.load_state(info["engine"])
        obs.log(f"[client {k}] resumed {csnap} (round {info['round']}, Adam step {model.flat.step})")
    beat = Heartbeat(cp, f"client{k}", cfg.heartbeat_s)
    # model sync (server.py:76-77 / client.py:261-264): client 0 alone reads the coordinator's
    # global model from the store and broadcasts it over the client data group (RCCL over
    # xGMI on the GPU) -- one host transfer per round instead of one per client.  With a
    # quorum < 1 a dead client must not stall a collective, so every client reads the store.
    bcast = ctx.initialized and ctx.num_clients > 1 and ctx.data_group is not None and cfg.quorum >= 1.0
    if bcast or agg == "allreduce":
        selfcheck(ctx, log=obs.log)  # every client, before round 0 (the coordinator is not in the data group)
    if bcast:  # every client is in every round: the cache can be built cooperatively
        catalog.attach(eng, ctx)
    if k == 0:
        plane = {"backend": dist.get_backend(ctx.data_group) if bcast else "store",
                 "size": dist.get_world_size(ctx.data_group) if bcast else 1}
        cp.put_json("data_plane", plane)
        obs.log(f"[client 0] model sync: {plane}")
    last: Dict = {}
    while True:
        flag = cp.get(f"r{r}/go").decode()
        if flag == "2":
            # the run is over and the coordinator asks for the FINAL global model's validation:
            # the per-round metrics (as the reference's) are each client's LOCAL model after its
            # local epochs, before the mean; this one scores the aggregate itself
            local = model.flat.flat.detach().clone()  # the client keeps its own model afterwards
            before = _backbone_before(model, full)
            _receive_global(cp, r, model, ctx, full, bcast)
            _backbone_synced(model, full, before)
            eng.ensure_cache()
            va = eng.validate()
            cp.put_json(f"r{r}/final/{k}", {"client": k, **{m: float(v) for m, v in va.items()
                                                              if isinstance(v, (int, float))}})
            with torch.no_grad():
                model.flat.flat.copy_(local)
            # stay until the coordinator has read every report: the store may live in this
            # process (rank 0 of the launch), and its exit would cut the others' reports off
            try:
                cp.get(f"r{r}/final_ack", min(cfg.round_timeout_s, 300.0) + 30.0)
            except Exception as e:  # (a coordinator gone: nothing left to wait for)
                obs.log(f"[client {k}] final evaluation: no acknowledgement: {e}")
            break
        if flag != "1":
            break
        beat(force=True)
        before = _backbone_before(model, full)
        _receive_global(cp, r, model, ctx, full, bcast)
        _backbone_synced(model, full, before)
        theta_g = model.flat.flat.detach().clone() if secure is not None else None  # the round's global model
        eng.ensure_cache()  # after the broadcast every client is here: the collective build point
        eng.sigma = _maybe_dp(cfg, eng)
        eng.epoch = 0
        tr, va = {}, {}
        t_train = t_valid = 0.0
        for _ in range(cfg.total_epochs):  # Trainer(...).train(total_epochs) per round (client.py:283-284)
            t0 = time.perf_counter()
            tr = eng.train_epoch(step_hook=beat)
            beat()
            t1 = time.perf_counter()
            va = eng.validate()
            beat()
            t_train += t1 - t0
            t_valid += time.perf_counter() - t1
        meta = {"client": k, "n_train": len(shard.train), "train_s": t_train, "valid_s": t_valid,
                **{m: float(v) for m, v in {**tr, **va}.items() if isinstance(v, (int, float))}}
        up = _client_upload_tensor(model, cfg).clone()
        if cfg.round_artifacts:  # client.py:288 torch.save(model.state_dict(), "model.pt")
            sub = "" if ctx.num_clients == 1 else f"client{k}"
            ckpt.save_state_dict(os.path.join(_artifact_dir(cfg), sub, "model.pt"), model)
        beat(force=True)
        fault.before_upload(r, up)
        if agg == "allreduce":
            w = float(len(shard.train)) if cfg.weighted_fedavg else 1.0
            wt = torch.tensor([w], device=up.device, dtype=torch.float32)
            up.mul_(wt)
            ipc = data_ipc(ctx, cfg.collective_timeout_s) if ctx.device.type == "cuda" else None
            comm.allreduce_([up, wt], ctx.data_group, ipc=ipc)
            if ipc is not None:
                ipc.check()
            up.div_(wt)
            if k == 0:
                cp.put_tensor(f"r{r}/avg", up.cpu())
            cp.put_json(f"r{r}/meta/{k}", meta)
        else:
            if secure is not None:
                # exact: the weighted delta on the grid the masked exponent histogram agrees
                w = float(len(shard.train)) if cfg.weighted_fedavg else 1.0
                meta.update(secure.upload(r, up, theta_g, w))
            else:
                cp.put_tensor(f"r{r}/up/{k}", up.cpu())
            cp.put_json(f"r{r}/meta/{k}", meta)
        if csnap:
            # after the upload (off the round's critical path), EVERY round, and only what a
            # resume needs: trainable flat + Adam + RNG + engine counters (~14 MB, not the 270 MB
            # full state with the frozen backbone).  Every round, not every save_every: a resume
            # from an older round would redraw the LDP noise / dropout of the rounds in between
            # at the same offsets, and noise that was already uploaded must never be reused
            ckpt.save_client_state(csnap, model, r, eng.state())
        last = meta
        r += 1
    _dump_flat(model, ctx)
    return last


def _flat_backbone(model: FedRecModel) -> torch.Tensor:
    ps = [p.detach().reshape(-1).float().cpu() for p in model.parameters() if not p.requires_grad]
    return torch.cat(ps) if ps else torch.zeros(0)


def _receive_global(cp, r: int, model: FedRecModel, ctx: DistContext, full: bool, bcast: bool) -> None:
    """Round ``r``'s global model into ``model`` (trainable flat buffer; + frozen backbone with
    ``sync=full``): from the store, or read by client 0 and RCCL-broadcast to the others."""
    if not bcast or ctx.client_index == 0:
        g = cp.get_tensor(f"r{r}/global")
        with torch.no_grad():
            model.flat.flat.copy_(g.to(model.flat.flat.device))
        if full:
            _load_flat_backbone(model, cp.get_tensor(f"r{r}/backbone"))
    if bcast:
        frozen = [p.data for p in model.parameters() if not p.requires_grad] if full else []
        with obs.range("model_broadcast"):
            comm.broadcast_([model.flat.flat, *frozen], src=ctx.client_ranks[0], group=ctx.data_group)


def _load_flat_backbone(model: FedRecModel, flat: torch.Tensor) -> None:
    o = 0
    with torch.no_grad():
        for p in model.parameters():
            if not p.requires_grad:
                n = p.numel()
                p.copy_(flat[o:o + n].view_as(p))
                o += n


def run_star_server(cfg: FedRecConfig, ctx: DistContext, run_id: str = "star") -> Dict:
    """Coordinator: holds the global model on the host (it never trains -- C20's
    ServerUserModel is only a parameter container; here it is the flat buffer)."""
    cp = ControlPlane.from_default(run_id, cfg.round_timeout_s)
    W = ctx.num_clients
    model = build_model(cfg, torch.device("cpu"))
    server = ServerStep.from_cfg(cfg)  # off by default: the plain mean
    start_round = 0
    if cfg.snapshot_path and os.path.exists(cfg.snapshot_path):
        info = ckpt.load_snapshot(cfg.snapshot_path, model)
        server.load(info.get("server_opt"))
        start_round = int(info.get("round") or 0) + 1 if info.get("round") is not None else 0
        obs.log(f"[server] resuming at round {start_round}")
    writer = _metrics_writer(cfg, True)
    agg = _aggregation(cfg, ctx)
    need = max(1, int(math.ceil(cfg.quorum * W)))
    full = cfg.sync == "full"
    hist = []
    cp.set("start", str(start_round))
    for r in range(start_round, cfg.global_rounds):
        t0 = time.perf_counter()
        cp.put_tensor(f"r{r}/global", model.flat.flat)
        if full:
            cp.put_tensor(f"r{r}/backbone", _flat_backbone(model))
        cp.set(f"r{r}/go", "1")
        dead: List[int] = []
        if agg == "allreduce":
            avg = cp.get_tensor(f"r{r}/avg", cfg.round_timeout_s)
            metas = [cp.get_json(f"r{r}/meta/{k}") for k in range(W)]
            accepted = list(range(W))
            new = avg
        else:
            keys = {k: f"r{r}/up/{k}" for k in range(W)}
            present, dead = cp.wait_uploads(keys, need, cfg.round_timeout_s, cfg.heartbeat_timeout_s,
                                            log=lambda m: obs.log(f"[server] round {r}: {m}"))
            ups, metas, accepted = [], [], []
            for key in present:
                k = int(key.rsplit("/", 1)[1])
                try:
                    t = cp.get_tensor(key)
                    meta = cp.get_json(f"r{r}/meta/{k}", 30.0)
                except Exception as e:  # corrupt blob / missing meta -> drop this client
                    obs.log(f"[server] round {r}: dropping client {k}: {e}")
                    continue
                if not cfg.secagg.enabled and not torch.isfinite(t).all():
                    obs.log(f"[server] round {r}: client {k} sent non-finite parameters; rejected")
                    continue
                ups.append(t)
                metas.append(meta)
                accepted.append(k)
                if cfg.round_artifacts and not cfg.secagg.enabled:  # server.py:27 received_model_{k}.pt
                    ckpt.atomic_save(ckpt.flat_to_state_dict(model, t),
                                     os.path.join(_artifact_dir(cfg), f"received_model_{k}.pt"))
            if cfg.secagg.enabled and len(accepted) != W:
                raise RuntimeError(f"secure aggregation needs every client (got {len(accepted)}/{W})")
            if len(accepted) < need:
                raise RuntimeError(f"round {r}: quorum not reached ({len(accepted)}/{W} < {need}); aborting")
            weights = [float(m["n_train"]) if cfg.weighted_fedavg else 1.0 for m in metas]
            if cfg.secagg.enabled:
                # the clients uploaded (w_k / sum w)(theta_k - theta_g) on the agreed grid: the
                # unmasked sum IS the FedAvg update (secagg.StarSecureUpload)
                new, fb = secagg.star_secure_aggregate(cp, r, W, ups, model.flat.flat.detach())
                if new is None:
                    obs.log(f"[server] round {r}: a client's update is non-finite; the global model is kept")
                    new = model.flat.flat.detach().clone()
            else:
                acc = torch.zeros_like(ups[0], dtype=torch.float64)
                for t, w in zip(ups, weights):
                    acc += t.double() * w  # server.py:46-50 (unweighted unless weighted_fedavg)
                new = (acc / sum(weights)).float()
        last_accepted = list(accepted)
        with torch.no_grad():
            if server.active:  # FedAvgM / server learning rate / FedAdam on the round's mean (fp64)
                new = server.apply(model.flat.flat.detach().double(), new.double()).float()
            model.flat.flat.copy_(new)
        dt = time.perf_counter() - t0
        rec = {"round": r, "clients_accepted": len(accepted), "clients": W, "clients_dead": dead, "round_s": dt}
        for key in ("training_loss", "validation_loss", "valid_auc", "valid_mrr", "val_ndcg@5", "val_ndcg@10",
                    "train_s", "valid_s"):
            vals = [m[key] for m in metas if key in m]
            if vals:
                rec[key] = float(np.mean(vals))
        imps = sum(m.get("impressions", 0.0) for m in metas)
        rec["impressions_per_s"] = imps / max(dt, 1e-9)
        writer.write(rec)
        hist.append(rec)
        obs.log(f"[server] round {r}: {len(accepted)}/{W} clients, {dt:.2f}s, auc={rec.get('valid_auc', float('nan')):.4f}")
        if cfg.snapshot_path:
            ckpt.save_snapshot(cfg.snapshot_path, model, r, round_idx=r, optim=False, config=cfg.to_dict(),
                               server_opt=server.state())
            gpath = os.path.join(os.path.dirname(os.path.abspath(cfg.snapshot_path)), f"global_model_round{r}.pt")
            ckpt.save_state_dict(gpath, model)
    R = max(cfg.global_rounds, start_round)
    if hist:
        # the final global model, validated by the clients on their validation shards (flag "2":
        # receive, validate, report, stop) -- the per-round records score each client's LOCAL
        # model after its local epochs, as the reference's Trainer.validate does (client.py:149-171)
        cp.put_tensor(f"r{R}/global", model.flat.flat)
        if full:
            cp.put_tensor(f"r{R}/backbone", _flat_backbone(model))
        cp.set(f"r{R}/go", "2")
        finals = []
        for k in last_accepted:  # (a client declared dead or dropped in the last round is not asked)
            try:
                finals.append(cp.get_json(f"r{R}/final/{k}", min(cfg.round_timeout_s, 300.0)))
            except Exception as e:  # a client gone after the last round: report the others
                obs.log(f"[server] final evaluation: no report from client {k}: {e}")
        cp.set(f"r{R}/final_ack", "1")  # the clients may exit now
        if finals:
            rec = {"round": R - 1, "final_global": True, "clients_reporting": len(finals)}
            for key in ("validation_loss", "valid_auc", "valid_mrr", "val_ndcg@5", "val_ndcg@10"):
                vals = [f[key] for f in finals if key in f]
                if vals:
                    rec[f"global_{key}"] = float(np.mean(vals))
            writer.write(rec)
            hist[-1].update({k2: v for k2, v in rec.items() if k2.startswith("global_")})
            obs.log(f"[server] final global model: auc={rec.get('global_valid_auc', float('nan')):.4f}")
    else:
        cp.set(f"r{R}/go", "0")  # server.py:105 stop flag
    return hist[-1] if hist else {}
