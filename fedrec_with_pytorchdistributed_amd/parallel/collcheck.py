"""Collective-sequence checker (the reference has no race/deadlock tooling).

A rank that issues a different sequence of data-plane collectives than its peers -- one
extra all-reduce, a bucket of another size or dtype, a skipped broadcast -- hangs RCCL or,
worse, silently sums mismatched buffers.  With ``FEDREC_COLL_CHECK=1`` every data-plane call
site records ``(op, dtype, numel, tag)`` into a running sha256 per rank; at epoch boundaries
``verify`` all-gathers (count, digest, last records) over the gloo control group and raises
:class:`CollectiveMismatch` on every rank, naming the first record where the ranks part.
Off by default: ``record`` is then a single attribute test.
"""
from __future__ import annotations

import hashlib
import os
from collections import deque
from typing import Deque, List, Optional, Tuple

import torch
import torch.distributed as dist


class CollectiveMismatch(RuntimeError):
    pass


class CollectiveChecker:
    def __init__(self, enabled: Optional[bool] = None, keep: int = 64):
        self.enabled = os.environ.get("FEDREC_COLL_CHECK", "0") == "1" if enabled is None else enabled
        self.keep = keep
        self.reset()

    def reset(self) -> None:
        self.count = 0
        self._h = hashlib.sha256()
        self.recent: Deque[Tuple[int, str]] = deque(maxlen=self.keep)

    def record(self, op: str, t: Optional[torch.Tensor] = None, tag: str = "") -> None:
        if not self.enabled:
            return
        # a call captured into a HIP graph runs once per REPLAY, not here: the replaying code
        # records it (train/engine.py _graph_step); ranks capture different numbers of graphs
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return
        meta = f"{op}|{str(t.dtype).replace('torch.', '')}|{t.numel()}" if t is not None else op
        rec = f"{meta}|{tag}"
        self.count += 1
        self._h.update(rec.encode())
        self._h.update(b"\0")
        self.recent.append((self.count, rec))

    def digest(self) -> str:
        return self._h.hexdigest()

    def verify(self, group=None, where: str = "") -> None:
        """Collective over ``group`` (every member must call it); raises on divergence."""
        if not self.enabled or not dist.is_available() or not dist.is_initialized():
            return
        world = dist.get_world_size(group)
        mine = (dist.get_rank(), self.count, self.digest(), list(self.recent))
        allv: List = [None] * world
        dist.all_gather_object(allv, mine, group=group)
        if len({d for _, _, d, _ in allv}) <= 1:
            return
        raise CollectiveMismatch(self.report(allv, where))

    @staticmethod
    def report(allv: List, where: str) -> str:
        lines = [f"collective sequences diverged{' at ' + where if where else ''}:"]
        for rank, n, d, _ in allv:
            lines.append(f"  rank {rank}: {n} collectives, digest {d[:16]}")
        # first index (within the kept window) where the recorded ops differ
        tables = [dict(rec) for _, _, _, rec in allv]
        common = set.intersection(*(set(t) for t in tables)) if tables else set()
        for i in sorted(common):
            vals = [t[i] for t in tables]
            if len(set(vals)) > 1:
                lines.append(f"  first difference at collective #{i}: " +
                             "; ".join(f"rank {r}: {v}" for (r, _, _, _), v in zip(allv, vals)))
                break
        else:
            counts = [n for _, n, _, _ in allv]
            lines.append(f"  kept window agrees; counts differ ({counts}) or the split is older than "
                         f"the last records")
        return "\n".join(lines)


CHECK = CollectiveChecker()
