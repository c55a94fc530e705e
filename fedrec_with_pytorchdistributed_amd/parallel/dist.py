"""Process groups: one process per GPU, roles decided by the entrypoint (not by rank).

* **data plane** -- RCCL (PyTorch's ``nccl`` backend on ROCm) over the client GPUs: the
  flat trainable bucket (4.66 MB fp32) is all-reduced / broadcast in ONE call, replacing
  the reference's 116 per-tensor gloo messages (``server.py:76-77``) and DDP buckets;
* **control plane** -- gloo on the host over *every* participant (coordinator + clients):
  round flags, role discovery, sample counts, metrics, heartbeats.

Roles are exchanged with ``all_gather_object`` so the coordinator can be any rank (the
reference hard-codes ``src=1``, Q13).  On a CPU-only run both planes are gloo.

Collective timeouts default to minutes, not the reference's 2 days (``client.py:227``).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist

from .collcheck import CHECK


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    role: str = "client"
    roles: List[str] = field(default_factory=lambda: ["client"])
    ctrl_group: Optional[object] = None  # gloo, everybody
    data_group: Optional[object] = None  # RCCL (or gloo on CPU), clients only
    client_ctrl_group: Optional[object] = None  # gloo, clients only (IPC handle exchange)
    client_ranks: List[int] = field(default_factory=lambda: [0])
    initialized: bool = False

    @property
    def client_index(self) -> int:
        return self.client_ranks.index(self.rank) if self.rank in self.client_ranks else -1

    @property
    def num_clients(self) -> int:
        return len(self.client_ranks)

    @property
    def coordinator(self) -> Optional[int]:
        return self.roles.index("server") if "server" in self.roles else None

    def barrier(self, group=None) -> None:
        if self.initialized:
            dist.barrier(group=group or self.ctrl_group)


def _env_int(k: str, d: int) -> int:
    v = os.environ.get(k)
    return int(v) if v is not None else d


def init(role: str = "client", device: str = "auto", timeout_s: float = 600.0, gpu_offset: int = 0) -> DistContext:
    """``gpu_offset``: GPU index = LOCAL_RANK - offset (a one-torchrun star run puts the
    coordinator on local rank 0 and the clients on GPUs 0..W-1)."""
    world = _env_int("WORLD_SIZE", 1)
    rank = _env_int("RANK", 0)
    local_rank = _env_int("LOCAL_RANK", 0)
    cpu_only = os.environ.get("FEDREC_CPU_ONLY", "0") == "1"
    use_cuda = not cpu_only and ((device == "cuda") or (device == "auto" and torch.cuda.is_available()
                                                        and role == "client"))
    if use_cuda:
        gi = max(0, local_rank - gpu_offset)
        if os.environ.get("FEDREC_SHARE_GPU", "0") == "1":
            # rehearsal of the multi-client path on a box with fewer GPUs than ranks (tests
            # only: RCCL refuses two ranks on one device, so pair it with FEDREC_DATA_BACKEND=gloo)
            gi %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(gi)
        dev = torch.device("cuda", gi)
    else:
        dev = torch.device("cpu")
    ctx = DistContext(rank=rank, world=world, local_rank=local_rank, device=dev, role=role, roles=[role],
                      client_ranks=[0], initialized=False)
    if world == 1:
        return ctx
    timeout = datetime.timedelta(seconds=timeout_s)
    # every rank must pick the same backends: decided by the machine, not by this rank's role
    gpu_job = torch.cuda.is_available() and os.environ.get("FEDREC_CPU_ONLY", "0") != "1"
    backend = "cpu:gloo,cuda:nccl" if gpu_job else "gloo"
    # no device_id: that would make the default group initialise its RCCL communicator eagerly,
    # a collective the CPU coordinator of a star run never joins (hang); the RCCL data group
    # below is created among the GPU clients only and initialises on first use.
    dist.init_process_group(backend=backend, init_method="env://", timeout=timeout)
    ctx.initialized = True
    ctx.ctrl_group = dist.new_group(backend="gloo", timeout=timeout)
    roles: List[Optional[str]] = [None] * world
    dist.all_gather_object(roles, role, group=ctx.ctrl_group)
    ctx.roles = [str(r) for r in roles]
    ctx.client_ranks = [i for i, r in enumerate(ctx.roles) if r == "client"]
    data_backend = os.environ.get("FEDREC_DATA_BACKEND") or ("nccl" if gpu_job else "gloo")
    # every rank must call new_group, members or not
    ctx.data_group = dist.new_group(ranks=ctx.client_ranks, backend=data_backend, timeout=timeout)
    ctx.client_ctrl_group = dist.new_group(ranks=ctx.client_ranks, backend="gloo", timeout=timeout)
    return ctx


def selfcheck(ctx: DistContext, nbytes: int = 4 << 20, log=None) -> dict:
    """Data-plane self-check before any timed / training work at N > 1 clients: every client
    all-reduces (a) its client index + 1 as an exact int64 scalar and (b) a ``nbytes`` fp32
    buffer of ones over the DATA group (RCCL over xGMI on the GPU), and the sums must be exact
    (W (W + 1) / 2 and W everywhere).  A misconfigured group, a wrong device mapping or a
    transport fault fails loudly here instead of as a silently wrong average later.  Returns
    ``{backend, size, us_4MB}``; raises RuntimeError on a mismatch."""
    import time

    if not ctx.initialized or ctx.num_clients <= 1 or ctx.client_index < 0:
        return {}
    W, k = ctx.num_clients, ctx.client_index
    dev = ctx.device
    t = torch.tensor([k + 1], dtype=torch.int64, device=dev)
    buf = torch.ones(max(1, nbytes // 4), dtype=torch.float32, device=dev)
    dist.all_reduce(t, group=ctx.data_group)
    dist.all_reduce(buf, group=ctx.data_group)  # warm-up / connection set-up
    buf.fill_(1.0)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    dist.all_reduce(buf, group=ctx.data_group)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    us = (time.perf_counter() - t0) * 1e6
    got_ids = int(t.item())
    ok_ids = got_ids == W * (W + 1) // 2
    bad = int((buf != float(W)).sum().item())
    info = {"backend": dist.get_backend(ctx.data_group), "size": dist.get_world_size(ctx.data_group),
            "device": str(dev), "us_4MB": round(us, 1), "ok": ok_ids and bad == 0}
    if log is not None:
        log(f"[client {k}] data-plane self-check: {info}")
    if not info["ok"]:
        raise RuntimeError(f"data-plane self-check FAILED on client {k}: id sum {got_ids} (expected "
                           f"{W * (W + 1) // 2}), {bad} wrong elements of {buf.numel()} (expected {W})")
    return info


def shutdown(ctx: DistContext) -> None:
    if ctx.initialized and dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:
            pass


def make_ipc_allreduce(ctx: DistContext, timeout_s: float = 600.0, device_epoch: bool = False):
    """The custom peer-to-peer all-reduce over IPC-mapped buffers among the client GPUs
    (:mod:`.ipc_allreduce`), or None (one client, no GPU).  ``device_epoch``: a capturable
    context (epochs counted on the device)."""
    if ctx.num_clients <= 1 or not ctx.initialized or ctx.device.type != "cuda" or ctx.client_index < 0:
        return None
    from .ipc_allreduce import IpcAllReduce

    return IpcAllReduce(ctx.client_ctrl_group, ctx.client_index, ctx.num_clients, ctx.device, timeout_s=timeout_s,
                        device_epoch=device_epoch)


def data_ipc(ctx: DistContext, timeout_s: float = 600.0):
    """The data plane's IPC all-reduce when ``FEDREC_ALLREDUCE=ipc`` selects it (one instance
    per context, shared by the GA bucket, the bucket reducer and parameter averaging), else
    None (RCCL).  Every client must make the same choice (the environment of the launch)."""
    if os.environ.get("FEDREC_ALLREDUCE", "rccl") != "ipc":
        return None
    ipc = getattr(ctx, "_ipc", None)
    if ipc is None:
        ipc = make_ipc_allreduce(ctx, timeout_s)
        ctx._ipc = ipc
    return ipc


def _ipc_grad_fn(ctx: DistContext, ipc, W: int):
    """The IPC all-reduce of the flat gradient.  ``split`` (set by the engine: the element offset
    where the user encoder's slice of the flat buffer starts, or None): the bucket goes as TWO
    calls, the user slice first -- the step graph issues that one early, on a side stream, as
    soon as the user encoder's weight gradients are final (DDP's first bucket), and the text-head
    slice after the backward (:meth:`finish_early`).  Eager steps issue the same two calls in the
    same order, so every client's sequence of calls on the context matches whichever path each
    step took."""

    def _ar_ipc(flat_grad: torch.Tensor) -> float:
        sp = _ar_ipc.split
        if sp:
            CHECK.record("all_reduce", flat_grad[sp:], "grad-ipc-user")
            ipc.allreduce_(flat_grad[sp:])
            CHECK.record("all_reduce", flat_grad[:sp], "grad-ipc-head")
            ipc.allreduce_(flat_grad[:sp])
        else:
            CHECK.record("all_reduce", flat_grad, "grad-ipc")
            ipc.allreduce_(flat_grad)
        return 1.0 / W

    def early(flat_grad: torch.Tensor, side: torch.cuda.Stream) -> None:
        """The user slice's call on ``side``, forked from the current stream (inside a capture:
        a graph branch beside the rest of the backward)."""
        main = torch.cuda.current_stream(flat_grad.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            ipc.allreduce_(flat_grad[_ar_ipc.split:])

    def finish_early(flat_grad: torch.Tensor, side: torch.cuda.Stream) -> float:
        """After :func:`early`: join the side stream, then the text-head slice's call."""
        torch.cuda.current_stream(flat_grad.device).wait_stream(side)
        ipc.allreduce_(flat_grad[:_ar_ipc.split])
        return 1.0 / W

    _ar_ipc.split = None
    _ar_ipc.early = early
    _ar_ipc.finish_early = finish_early
    _ar_ipc.check = ipc.check
    _ar_ipc.kind = "ipc"
    # device epochs: the launch is capturable -- the engine puts it inside the step graph, between
    # the backward and the device-step Adam (one replay per step at N > 1, as at N = 1)
    _ar_ipc.capturable = True
    _ar_ipc.ipc = ipc
    return _ar_ipc


def _rccl_grad_fn(ctx: DistContext, W: int):
    def _ar(flat_grad: torch.Tensor) -> float:
        CHECK.record("all_reduce", flat_grad, "grad")
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=ctx.data_group)
        return 1.0 / W

    _ar.kind = "rccl" if ctx.device.type == "cuda" else dist.get_backend(ctx.data_group)
    # the library path stays eager (on the optimizer side stream, after the step graph): the
    # capturable all-reduce of the step graph is the device-epoch IPC one
    _ar.capturable = False
    return _ar


def probe_ipc_grad(ctx: DistContext, nelem: int, timeout_s: float = 600.0, check_timeout_s: float = 20.0,
                   reps: int = 10, log=None) -> dict:
    """Set up the device-epoch IPC all-reduce for the gradient bucket and check it against the
    data group's sum (RCCL on the node) on an ``nelem`` fp32 bucket, timing both (eager, ``reps``
    calls).  The verdict is agreed by every client (gloo MIN / MAX).  Returns ``{"ok", "ipc_ms",
    "group_ms", "ipc": IpcAllReduce or None}``; a failure (an exception, a wrong sum, a peer that
    never arrives within ``check_timeout_s``) gives ok False and no context."""
    import time

    info = {"ok": False, "ipc_ms": None, "group_ms": None, "ipc": None}
    ipc = None
    ok = 1
    ms = [0.0, 0.0]

    def _fail(e):  # pragma: no cover - depends on the node
        if log is not None:
            log(f"[client {ctx.client_index}] IPC all-reduce probe failed: {e!r}"[:400])
        return 0

    try:
        ipc = make_ipc_allreduce(ctx, timeout_s=check_timeout_s, device_epoch=True)
        dev = ctx.device
        a = torch.randn(nelem, device=dev, generator=torch.Generator(dev).manual_seed(1234 + ctx.client_index))
        b = a.clone()
        dist.all_reduce(a, group=ctx.data_group)
        ipc.allreduce_(b)
        torch.cuda.synchronize(dev)
        ok = int(ipc.status() == 0 and bool(torch.allclose(a, b, rtol=1e-5, atol=1e-5)))
    except Exception as e:  # pragma: no cover - depends on the node
        ok = _fail(e)
    # agree on correctness BEFORE any timing collective: every client then runs the same sequence
    # of control-group calls (a client that failed alone must not skip the barriers below)
    t = torch.tensor([ok], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.client_ctrl_group)
    if int(t.item()):
        for k, fn in enumerate((lambda x: ipc.allreduce_(x), lambda x: dist.all_reduce(x, group=ctx.data_group))):
            try:
                fn(b)
                torch.cuda.synchronize(dev)
            except Exception as e:  # pragma: no cover
                ok = _fail(e)
            dist.barrier(group=ctx.client_ctrl_group)
            if not ok:
                continue
            try:
                t0 = time.perf_counter()
                for _ in range(reps):
                    fn(b)
                torch.cuda.synchronize(dev)
                ms[k] = 1000.0 * (time.perf_counter() - t0) / reps
            except Exception as e:  # pragma: no cover
                ok = _fail(e)
        try:
            ok = int(ok and ipc.status() == 0)
        except Exception as e:  # pragma: no cover
            ok = _fail(e)
        t = torch.tensor([ok], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.client_ctrl_group)
    tm = torch.tensor(ms, dtype=torch.float64)
    dist.all_reduce(tm, op=dist.ReduceOp.MAX, group=ctx.client_ctrl_group)
    info["ok"] = bool(t.item())
    info["ipc_ms"], info["group_ms"] = round(float(tm[0]), 4), round(float(tm[1]), 4)
    if info["ok"]:
        ipc.timeout_s = float(timeout_s)  # the run's collective timeout from here on
        info["ipc"] = ipc
    elif ipc is not None:
        try:
            ipc.close()
        except Exception:  # pragma: no cover
            pass
    return info


def make_grad_allreduce(ctx: DistContext, timeout_s: float = 600.0, choice: Optional[str] = None, log=None,
                        nelem: int = 1 << 20):
    """Sum the flat gradient over the client data group; returns the 1/W scale Adam applies.

    ``choice`` (default: ``FEDREC_ALLREDUCE``, else ``rccl``):
      * ``rccl`` -- ``dist.all_reduce`` on the data group (RCCL over xGMI; gloo on the CPU);
      * ``ipc``  -- the custom IPC all-reduce with device epochs: capturable, so the engine runs
        it INSIDE the step graph (every rank gets the bitwise-same sum); its ``check`` (run by
        the engine at every epoch end) raises if a peer timed out;
      * ``auto`` -- ``ipc`` when :func:`probe_ipc_grad` finds it correct on this node and not
        slower than the data group's all-reduce by more than 25 % (isolated, eager), else ``rccl``.
    ``nelem``: the bucket the probe checks and times (the flat gradient's size).  The returned
    callable carries ``kind``, ``capturable`` and (auto) ``probe``."""
    if ctx.num_clients <= 1 or not ctx.initialized:
        return None
    W = ctx.num_clients
    choice = choice or os.environ.get("FEDREC_ALLREDUCE", "rccl")
    if ctx.device.type != "cuda" or choice not in ("ipc", "auto"):
        return _rccl_grad_fn(ctx, W)
    if choice == "ipc":
        return _ipc_grad_fn(ctx, make_ipc_allreduce(ctx, timeout_s, device_epoch=True), W)
    probe = probe_ipc_grad(ctx, int(nelem), timeout_s=timeout_s, log=log)
    use = probe["ok"] and probe["ipc_ms"] <= 1.25 * probe["group_ms"]
    fn = _ipc_grad_fn(ctx, probe["ipc"], W) if use else _rccl_grad_fn(ctx, W)
    if not use and probe["ipc"] is not None:
        probe["ipc"].close()
    fn.probe = {k: v for k, v in probe.items() if k != "ipc"}
    return fn


def make_secure_grad_allreduce(ctx: DistContext, timeout_s: float = 600.0, run_id: str = "secagg-ga"):
    """Gradient averaging under pairwise-mask secure aggregation (BASELINE config 5).

    Each client uploads ``Q(g) + sum_j +-PRG(s_ij, step)`` as wrap-around int32; one RCCL
    int32 SUM all-reduce cancels the masks exactly; the result is dequantised in place.
    Pair seeds come from a Diffie-Hellman exchange of public keys over the store.  The
    fixed-point bound is agreed per step by a masked exponent histogram
    (:class:`.secagg.ExactMasker`): nothing is clamped, no host read."""
    from . import secagg
    from .control import ControlPlane

    if ctx.num_clients <= 1 or not ctx.initialized:
        return None
    W, k = ctx.num_clients, ctx.client_index
    cp = ControlPlane.from_default(run_id, timeout_s)
    kp = secagg.KeyPair()
    cp.set(f"pk/{k}", secagg.public_bytes(kp))
    pubs = [cp.get(f"pk/{j}") for j in range(W)]
    seeds_row = secagg.seeds_from_publics(kp, k, pubs)
    masker = secagg.ExactMasker(k, W, seeds_row, ctx.device)
    ipc = data_ipc(ctx, timeout_s) if ctx.device.type == "cuda" else None
    state = {"step": 0}

    def _ar(flat_grad: torch.Tensor) -> float:
        masker.allreduce_(flat_grad, state["step"], ctx.data_group, "secagg", ipc=ipc)
        state["step"] += 1
        return 1.0 / W

    if ipc is not None:
        _ar.check = ipc.check
    return _ar


def make_bucket_reducer(ctx: DistContext, flat, secure: bool = False, bucket_mb: Optional[float] = None,
                        timeout_s: float = 600.0, run_id: str = "secagg-bucket"):
    """The backward-overlapped bucketed all-reduce (:class:`.reducer.BucketReducer`) over the
    client data group; ``secure`` = pairwise-masked int32 buckets (seeds by Diffie-Hellman
    over the store, as :func:`make_secure_grad_allreduce`).  None for a single client."""
    from .reducer import DEFAULT_BUCKET_MB, BucketReducer

    if ctx.num_clients <= 1 or not ctx.initialized:
        return None
    W, k = ctx.num_clients, ctx.client_index
    seeds_row = None
    if secure:
        from . import secagg
        from .control import ControlPlane

        cp = ControlPlane.from_default(run_id, timeout_s)
        kp = secagg.KeyPair()
        cp.set(f"pk/{k}", secagg.public_bytes(kp))
        seeds_row = secagg.seeds_from_publics(kp, k, [cp.get(f"pk/{j}") for j in range(W)])
    mb = float(os.environ.get("FEDREC_BUCKET_MB", bucket_mb or DEFAULT_BUCKET_MB))
    ipc = data_ipc(ctx, timeout_s) if ctx.device.type == "cuda" else None
    return BucketReducer(flat, ctx.data_group, W, "secure" if secure else "mean", mb, k, seeds_row, ipc=ipc)
