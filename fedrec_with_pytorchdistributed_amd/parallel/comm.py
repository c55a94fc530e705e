"""Data-plane collectives over the client group (RCCL on GPUs, gloo on CPU).

Bucket sizing for xGMI: the trainable set is ONE 4.66 MB bucket (it is
already a single flat buffer, so no pack/unpack copy).  Larger syncs (``sync=full``, Q15:
the reference all-reduces all 116 tensors = 270 MB every epoch) are cut into ~28 MB
buckets = 8 ranks x 7 links x 512 KB, so every per-peer xGMI transfer stays >= 512 KB
while several buckets can be in flight.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from .collcheck import CHECK

BUCKET_BYTES = 28 << 20


def _buckets(tensors: List[torch.Tensor], bucket_bytes: int):
    cur, size = [], 0
    for t in tensors:
        nb = t.numel() * t.element_size()
        if cur and (size + nb > bucket_bytes or t.dtype != cur[0].dtype or t.device != cur[0].device):
            yield cur
            cur, size = [], 0
        cur.append(t)
        size += nb
    if cur:
        yield cur


def allreduce_(tensors: List[torch.Tensor], group, op=dist.ReduceOp.SUM, scale: Optional[float] = None,
               bucket_bytes: int = BUCKET_BYTES, ipc=None) -> None:
    """In-place all-reduce of ``tensors`` in ~28 MB buckets (async, all in flight); ``scale``
    multiplies the result (the 1/W of a mean).  ``ipc`` (:func:`.dist.data_ipc`, fp32 SUM on the
    device): the custom IPC all-reduce moves each bucket instead of ``group``."""
    if ipc is not None and op == dist.ReduceOp.SUM and all(t.is_cuda and t.dtype == torch.float32 for t in tensors):
        for b in _buckets(tensors, bucket_bytes):
            flat = b[0] if (len(b) == 1 and b[0].is_contiguous()) else _flatten_dense_tensors(b)
            CHECK.record("all_reduce", flat, "SUM")
            ipc.allreduce_(flat)
            if scale is not None:
                flat.mul_(scale)
            if len(b) == 1:
                if flat.data_ptr() != b[0].data_ptr():
                    b[0].copy_(flat.view_as(b[0]))
            else:
                for t, s in zip(b, _unflatten_dense_tensors(flat, b)):
                    t.copy_(s)
        return
    works = []
    for b in _buckets(tensors, bucket_bytes):
        if len(b) == 1:
            flat = b[0] if b[0].is_contiguous() else b[0].contiguous()
            CHECK.record("all_reduce", flat, str(op).split(".")[-1])
            works.append((b, flat, dist.all_reduce(flat, op=op, group=group, async_op=True)))
        else:
            flat = _flatten_dense_tensors(b)
            CHECK.record("all_reduce", flat, str(op).split(".")[-1])
            works.append((b, flat, dist.all_reduce(flat, op=op, group=group, async_op=True)))
    for b, flat, w in works:
        w.wait()
        if scale is not None:
            flat.mul_(scale)
        if len(b) == 1:
            if flat.data_ptr() != b[0].data_ptr():
                b[0].copy_(flat.view_as(b[0]))
        else:
            for t, s in zip(b, _unflatten_dense_tensors(flat, b)):
                t.copy_(s)


def broadcast_(tensors: List[torch.Tensor], src: int, group, bucket_bytes: int = BUCKET_BYTES) -> None:
    for b in _buckets(tensors, bucket_bytes):
        if len(b) == 1 and b[0].is_contiguous():
            CHECK.record("broadcast", b[0], f"src={src}")
            dist.broadcast(b[0], src=src, group=group)
        else:
            flat = _flatten_dense_tensors(b)
            CHECK.record("broadcast", flat, f"src={src}")
            dist.broadcast(flat, src=src, group=group)
            for t, s in zip(b, _unflatten_dense_tensors(flat, b)):
                t.copy_(s)
