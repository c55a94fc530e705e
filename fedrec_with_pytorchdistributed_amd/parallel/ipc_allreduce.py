"""Custom peer-to-peer all-reduce over IPC-mapped device buffers (``csrc/ipc_allreduce.hip``).

SURVEY §5.8.2 / §7.3 P6: the data plane's gradient and parameter buckets (4.66 MB trainable set;
~28 MB buckets of the unfrozen config) are small enough that a ring all-reduce is latency-bound
on a node whose GPUs are fully connected by xGMI.  Here every client exports one uncached
device region (hipIpcGetMemHandle), the handles travel over the gloo control group, and each
call runs ONE kernel per rank:

* ``one-shot`` (buckets up to ``one_shot_max``): publish the input, one cross-rank barrier
  (release / acquire flags in the peers' regions), every rank reads all W inputs over xGMI and
  sums them in rank order -- every rank gets the bitwise-same result.
* ``two-shot`` (larger buckets): reduce-scatter of 1/W slices, barrier, all-gather of the
  reduced slices: 2 (W-1)/W of the bucket read per rank instead of (W-1).

fp32 SUM and int32 wrap-around SUM (the pairwise-masked fixed point of secure aggregation).
RCCL stays the default data plane; ``FEDREC_ALLREDUCE=ipc`` selects this one for the GA flat
bucket, the unfrozen / secure bucket reducer and parameter averaging, and the bench reports both
at N > 1.  The barrier waits are bounded by the collective timeout: a missing peer makes the
kernel record a timeout in its status word, poison its output and exit instead of hanging the
GPU, and :meth:`IpcAllReduce.check` (run by the engine at every epoch end) raises on it.

Reference call sites this replaces: ``Gradient_Averaging_main.py:119`` (DDP reducer),
``Parameter_Averaging_main.py:144-148`` (per-tensor parameter all-reduce).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import native

DEFAULT_CAP = 32 << 20  # bytes per slot (two slots + flags per rank)


class IpcAllReduce:
    """One rank's end of the IPC all-reduce among the ``world`` clients of ``ctrl_group``."""

    def __init__(self, ctrl_group, rank: int, world: int, device: torch.device, cap: int = DEFAULT_CAP,
                 one_shot_max: Optional[int] = None, blocks: Optional[int] = None, timeout_s: float = 600.0,
                 device_epoch: bool = False):
        """``device_epoch``: every call's epoch comes from a device counter of the context (the
        launch is capturable in a HIP graph: each replay runs the next epoch); such a context
        takes device-epoch calls only."""
        self.lib = native.lib()
        self.rank, self.world, self.device = int(rank), int(world), device
        self.device_epoch = bool(device_epoch)
        if one_shot_max is None:
            # one-shot reads (W - 1) buckets per rank, two-shot 2 (W - 1) / W of one plus a second
            # barrier: one-shot for two ranks, two-shot for larger groups past 512 KB
            one_shot_max = (8 << 20) if world <= 2 else (512 << 10)
        if blocks is None:
            blocks = 32
        self.cap, self.one_shot_max, self.blocks = int(cap), int(one_shot_max), int(blocks)
        self.timeout_s = float(timeout_s)
        self.id = None
        hb = None
        try:
            with torch.cuda.device(device):
                self.id, h = self.lib.ipc_create(self.cap)
            hb = bytes(h.numpy().tobytes())
        except RuntimeError:  # reported below, after every rank has joined the exchange
            pass
        # every rank must run the same protocol geometry (the barrier waits on blocks x ranks
        # flags; a different one-shot threshold would split one call into different modes)
        geo = (self.cap, self.one_shot_max, self.blocks)
        handles: List[Optional[tuple]] = [None] * self.world
        dist.all_gather_object(handles, (hb, geo), group=ctrl_group)
        if any(g[0] is None for g in handles) or any(g[1] != geo for g in handles):
            if self.id is not None:
                self.lib.ipc_destroy(self.id)
                self.id = None
            raise RuntimeError(f"IPC all-reduce: a rank could not create its region, or the ranks disagree on "
                               f"(cap, one_shot_max, blocks): {[(g[0] is not None, g[1]) for g in handles]}")
        flat = torch.frombuffer(bytearray(b"".join(g[0] for g in handles)), dtype=torch.uint8)
        err = None
        try:
            with torch.cuda.device(device):
                self.lib.ipc_open(self.id, flat, self.rank, self.world, None)
        except RuntimeError as e:  # (a peer's region could not be mapped here)
            err = e
        # every rank learns whether every rank opened every region (one gloo MIN) -- a rank that
        # failed must not leave the others waiting in a barrier or, worse, in a kernel
        ok = torch.tensor([0 if err is not None else 1], dtype=torch.int64)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=ctrl_group)
        if int(ok.item()) == 0:
            self.lib.ipc_destroy(self.id)
            self.id = None
            raise RuntimeError(f"IPC all-reduce: a rank could not open the peers' regions"
                               + (f" (here: {err})" if err is not None else " (on another rank)"))
        self.epoch = 0

    def allreduce_(self, t: torch.Tensor, mode: Optional[str] = None) -> torch.Tensor:
        """In-place SUM of ``t`` (fp32 or int32, on this rank's device) over the ranks."""
        return _allreduce(self, t, mode)

    def status(self) -> int:
        """0 = every call completed; 1 = a barrier timed out (a peer never arrived).  Reads the
        device (synchronises with it)."""
        return int(self.lib.ipc_status(self.id))

    def status_word(self) -> torch.Tensor:
        """The status word as a device int32 [1] view (nonzero after a peer timeout): the
        in-graph Adam skips its update on it (a view of the context's allocation, valid until
        :meth:`close`)."""
        if getattr(self, "_status_word", None) is None:
            self._status_word = self.lib.ipc_status_word(self.id)
        return self._status_word

    def check(self) -> None:
        """Raise if any call since the start timed out (its output was poisoned); one device
        read -- the engine calls it at every epoch end, where it synchronises anyway."""
        if self.id is not None and self.status() != 0:
            raise RuntimeError(f"IPC all-reduce on client {self.rank}: a peer did not arrive within "
                               f"{self.timeout_s:.0f} s (the reduced gradients of that call are invalid)")

    def close(self) -> None:
        if self.id is not None:
            torch.cuda.synchronize(self.device)
            self._status_word = None
            self.lib.ipc_destroy(self.id)
            self.id = None


def _allreduce(g, t: torch.Tensor, mode: Optional[str]) -> torch.Tensor:
    if t.dtype not in (torch.float32, torch.int32):
        raise TypeError(f"IPC all-reduce: fp32 / int32 only, got {t.dtype}")
    nbytes = t.numel() * 4
    if nbytes > g.cap:
        # larger than one slot: consecutive chunks (each call a full barrier-protected epoch)
        src = t if t.is_contiguous() else t.contiguous()
        flat = src.reshape(-1)
        step = (g.cap // 16) * 4
        for s in range(0, flat.numel(), step):
            _allreduce(g, flat[s:s + step], mode)
        if src is not t:
            t.copy_(src)
        return t
    work = t if (t.is_contiguous() and t.numel() % 4 == 0) else None
    if work is None:  # pad to whole 16-byte chunks (the kernel moves float4 / int4)
        work = torch.zeros(-(-t.numel() // 4) * 4, dtype=t.dtype, device=t.device)
        work[:t.numel()].copy_(t.reshape(-1))
    m = mode or ("one" if nbytes <= g.one_shot_max else "two")
    g.epoch += 1  # (a device-epoch context passes 0: the kernel takes its own counter + 1)
    g.lib.ipc_allreduce_(g.id, work.view(-1), 0 if getattr(g, "device_epoch", False) else g.epoch,
                         0 if m == "one" else 1, g.blocks, g.timeout_s)
    if work is not t:
        t.view(-1).copy_(work[:t.numel()])
    return t


class LocalIpcGroup:
    """Single-process rehearsal of the protocol: ``world`` ranks' regions on ONE device and ONE
    launch whose blocks play every rank (rank = block / blocks-per-rank), synchronising through
    the same per-rank flags, slots and barriers as the per-process kernels -- co-resident by
    construction (one kernel per rank on separate streams depends on the streams landing on
    distinct hardware queues).  Used by the 1-GPU tests; the multi-process form is
    :class:`IpcAllReduce`."""

    def __init__(self, world: int, device: torch.device, cap: int = 4 << 20, blocks: int = 8,
                 timeout_s: float = 60.0):
        lib = native.lib()
        self.timeout_s = float(timeout_s)
        self.lib, self.world, self.device, self.cap, self.blocks = lib, int(world), device, int(cap), int(blocks)
        self.one_shot_max = 1 << 62
        with torch.cuda.device(device):
            made = [lib.ipc_create(self.cap) for _ in range(self.world)]
        self.ids = [m[0] for m in made]
        regions = torch.tensor([lib.ipc_region(i) for i in self.ids], dtype=torch.int64)
        handles = torch.cat([m[1] for m in made])
        for r, i in enumerate(self.ids):
            lib.ipc_open(i, handles, r, self.world, regions)
        self.epoch = 0

    def allreduce_(self, ts: List[torch.Tensor], mode: str = "one") -> None:
        """``ts[r]`` = rank r's tensor; every one is replaced by the sum."""
        self.epoch += 1
        self.lib.ipc_allreduce_local_(self.ids, [t.view(-1) for t in ts], self.epoch, 0 if mode == "one" else 1,
                                      self.blocks, self.timeout_s)

    def status(self) -> List[int]:
        return [int(self.lib.ipc_status(i)) for i in self.ids]

    def close(self) -> None:
        torch.cuda.synchronize(self.device)
        for i in self.ids:
            self.lib.ipc_destroy(i)
        self.ids = []
