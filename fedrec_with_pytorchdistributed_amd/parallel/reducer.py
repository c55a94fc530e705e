"""Bucketed gradient all-reduce overlapped with the backward (the DDP reducer's job).

The reference wraps its model in DDP (``Gradient_Averaging_main.py:119``), whose reducer
all-reduces gradient buckets as the backward produces them.  Here the trainable gradients
live in one flat fp32 buffer (:class:`..models.fedrec_model.FlatParams`); this reducer cuts
it into contiguous buckets along parameter boundaries (~28 MB: SURVEY §5.8 item 3, 8 ranks x
7 xGMI links x 512 KB per-peer chunk), ordered as the backward fills them (last registered
parameter first), and on a dedicated communication stream reduces each bucket as soon as
every one of its parameters has its gradient -- while the backward of the earlier layers
still runs on the compute stream.

* ``op="mean"``: one RCCL SUM all-reduce per bucket (the 1/W lands in Adam's grad scale).
* ``op="secure"``: pairwise-masked fixed-point aggregation per bucket (BASELINE config 5,
  :class:`.secagg.ExactMasker`): a 1 KB masked exponent histogram agrees on a bound every
  client's values fit (nothing is clamped, at any number of clients), then ONE int32 SUM
  all-reduce of the bucket cancels the masks exactly.  Both run on the communication stream
  with no host read.

Parameters register ``post_accumulate_grad`` hooks: the hook copies the fresh gradient into
its flat slot, re-points ``.grad`` at the slot, and counts the bucket down.  A bucket whose
parameters got no gradient is reduced by :meth:`finish` (after ``FlatParams.end_backward``
zero-filled them), in bucket order, so every rank issues the same collective sequence.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from .collcheck import CHECK

DEFAULT_BUCKET_MB = 28.0


class BucketReducer:
    def __init__(self, flat, group, world: int, op: str = "mean", bucket_mb: float = DEFAULT_BUCKET_MB,
                 client_index: int = 0, seeds_row=None, ipc=None):
        if op not in ("mean", "secure"):
            raise ValueError(f"BucketReducer op {op!r}")
        self.flat, self.group, self.W, self.op = flat, group, int(world), op
        self.ipc = ipc  # parallel.ipc_allreduce.IpcAllReduce (FEDREC_ALLREDUCE=ipc), else RCCL / gloo
        self.k = client_index
        dev = flat.grad.device
        self.device = dev
        cap = max(1, int(bucket_mb * 2**20) // 4)
        # parameters in backward order (reverse registration) -> contiguous flat ranges
        order = list(range(len(flat.params)))[::-1]
        self.buckets: List[List[int]] = []
        cur, size = [], 0
        for i in order:
            n = flat.params[i].numel()
            if cur and size + n > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(i)
            size += n
        if cur:
            self.buckets.append(cur)
        self.ranges = []
        for b in self.buckets:
            lo = min(flat.offsets[i] for i in b)
            hi = max(flat.offsets[i] + flat.params[i].numel() for i in b)
            self.ranges.append((lo, hi))
        self.bucket_of = {i: bi for bi, b in enumerate(self.buckets) for i in b}
        self.comm = torch.cuda.Stream(dev) if dev.type == "cuda" else None
        self.step = 0
        self._pending: List[int] = []
        self._launched: List[bool] = []
        self._active = False
        if op == "secure":
            from . import secagg

            self.maskers = [secagg.ExactMasker(self.k, self.W, seeds_row, dev) for _ in self.buckets]
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(flat.params)]

    # -------------------------------------------------------------------------------
    def begin(self) -> None:
        """Arm the reducer for one backward pass."""
        self._pending = [len(b) for b in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._active = True

    def _make_hook(self, i: int):
        def hook(p: torch.Tensor) -> None:
            if not self._active:
                return
            off, n = self.flat.offsets[i], p.numel()
            view = self.flat.grad[off:off + n].view_as(p)
            if p.grad is not None and p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad)
                p.grad = view
            b = self.bucket_of[i]
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._launch(b)
        return hook

    def _launch(self, b: int) -> None:
        if self._launched[b]:
            return
        self._launched[b] = True
        lo, hi = self.ranges[b]
        g = self.flat.grad[lo:hi]
        if self.comm is None:
            self._reduce(g, b)
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.comm.wait_event(ev)
        with torch.cuda.stream(self.comm):
            self._reduce(g, b)

    def _reduce(self, g: torch.Tensor, b: int) -> None:
        if self.op == "mean":
            CHECK.record("all_reduce", g, f"bucket{b}")
            if self.ipc is not None:
                self.ipc.allreduce_(g)
            else:
                dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group)
            return
        rnd = self.step * 4096 + b  # a fresh PRG counter space per (step, bucket)
        self.maskers[b].allreduce_(g, rnd, self.group, f"secagg{b}", ipc=self.ipc)

    def check(self) -> None:
        """Raise if an IPC all-reduce of this reducer timed out (engine: every epoch end)."""
        if self.ipc is not None:
            self.ipc.check()

    def finish(self) -> float:
        """Reduce any bucket still waiting (parameters without a gradient: zero-filled by
        ``end_backward``), make the compute stream wait for every bucket; returns 1/W.

        Without a :meth:`begin` (the ``per_epoch`` schedule accumulates several backward
        passes and reduces once, at the epoch-end optimizer step) every bucket is reduced
        here, in bucket order."""
        if not self._active:
            self._launched = [False] * len(self.buckets)
        for b in range(len(self.buckets)):
            if not self._launched[b]:
                self._launch(b)
        if self.comm is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.comm)
        self._active = False
        self.step += 1
        return 1.0 / self.W

    def close(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
