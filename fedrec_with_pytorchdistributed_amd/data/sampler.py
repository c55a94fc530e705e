"""Batch assembly: negative sampling + history padding (reference ``dataset.py:8-86``).

Train row ``[_, pos, negs, his, _]`` -> ``candidates = [pos] + newsample(negs, 4)``,
``history = ids + [0] * (50 - len)``, ``label = 0`` (the positive is always column 0):

* ``newsample`` (``dataset.py:10-14``): fewer than ``npratio`` negatives -> the negatives
  followed by ``<unk>`` (id 0) padding, in order; otherwise ``random.sample(negs, 4)``: a
  uniformly random ordered 4-subset.  Here it is seeded per (seed, rank, epoch) (Q16).
* History: the reference pads but never truncates (Q6, the shipped shard has 76 items);
  default keeps the most recent ``max_his_len`` items.  With
  ``compat.no_history_truncation`` the batch is padded to its longest history instead.

Validation (``client.py:158-165``): candidates ``[pos] + negs[-4:]`` (padded with 0 when a
row has fewer), same history rule.

Two implementations with identical semantics: :class:`HostSampler` (numpy, vectorised per
batch) and the device sampler in ``ops.sample_batch`` (HIP, the shard resident in HBM).
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import numpy as np

from .shard import ImpressionArrays


def _pad_history(arr: ImpressionArrays, rows: np.ndarray, max_his: int, truncate: bool) -> np.ndarray:
    lens = (arr.his_ptr[rows + 1] - arr.his_ptr[rows]).astype(np.int64)
    if truncate:
        H = max_his
        take = np.minimum(lens, H)
    else:
        H = max(max_his, int(lens.max()) if len(lens) else max_his)
        take = lens
    out = np.zeros((len(rows), H), dtype=np.int32)
    start = arr.his_ptr[rows + 1] - take  # most recent items (histories are chronological)
    j = np.arange(H)[None, :]
    valid = j < take[:, None]
    src = np.where(valid, start[:, None] + j, 0)
    out[valid] = arr.his_ids[src[valid]]
    return out


def train_candidates(arr: ImpressionArrays, rows: np.ndarray, npratio: int,
                     rng: np.random.Generator) -> np.ndarray:
    B = len(rows)
    nl = (arr.neg_ptr[rows + 1] - arr.neg_ptr[rows]).astype(np.int64)
    maxn = max(int(nl.max()) if B else 0, npratio)
    keys = rng.random((B, maxn))
    j = np.arange(maxn)[None, :]
    keys[j >= nl[:, None]] = np.inf
    pick = np.argsort(keys, axis=1, kind="stable")[:, :npratio]
    short = nl < npratio
    # rows with too few negatives: in order, then <unk> padding
    pick[short] = np.broadcast_to(np.arange(npratio), (int(short.sum()), npratio))
    valid = pick < nl[:, None]
    src = arr.neg_ptr[rows][:, None] + pick
    negs = np.where(valid, arr.neg_ids[np.where(valid, src, 0)], 0)
    cand = np.empty((B, npratio + 1), dtype=np.int32)
    cand[:, 0] = arr.pos[rows]
    cand[:, 1:] = negs
    return cand


def valid_candidates(arr: ImpressionArrays, rows: np.ndarray, npratio: int) -> np.ndarray:
    B = len(rows)
    nl = (arr.neg_ptr[rows + 1] - arr.neg_ptr[rows]).astype(np.int64)
    take = np.minimum(nl, npratio)
    j = np.arange(npratio)[None, :]
    start = arr.neg_ptr[rows + 1] - take
    valid = j < take[:, None]
    src = np.where(valid, start[:, None] + j, 0)
    cand = np.zeros((B, npratio + 1), dtype=np.int32)
    cand[:, 0] = arr.pos[rows]
    cand[:, 1:] = np.where(valid, arr.neg_ids[src], 0)
    return cand


class HostSampler:
    """Epoch iterator over a client's train impressions."""

    def __init__(self, arr: ImpressionArrays, batch_size: int, npratio: int = 4, max_his: int = 50,
                 truncate: bool = True, seed: int = 0, rank: int = 0, shuffle: bool = True,
                 drop_last: bool = False):
        self.arr, self.B, self.npratio, self.max_his = arr, batch_size, npratio, max_his
        self.truncate, self.seed, self.rank = truncate, seed, rank
        self.shuffle, self.drop_last = shuffle, drop_last

    def num_batches(self) -> int:
        n = len(self.arr)
        return n // self.B if self.drop_last else -(-n // self.B)

    def epoch(self, epoch: int) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
        rng = np.random.Generator(np.random.PCG64([self.seed, self.rank, epoch, 17]))
        n = len(self.arr)
        order = rng.permutation(n) if self.shuffle else np.arange(n)
        for b in range(self.num_batches()):
            rows = order[b * self.B:(b + 1) * self.B]
            yield self.batch(rows, rng)

    def batch(self, rows: np.ndarray, rng: np.random.Generator) -> Tuple[np.ndarray, np.ndarray]:
        cand = train_candidates(self.arr, rows, self.npratio, rng)
        his = _pad_history(self.arr, rows, self.max_his, self.truncate)
        return cand, his


def validation_batches(arr: ImpressionArrays, batch_size: int, npratio: int = 4, max_his: int = 50,
                       truncate: bool = True, limit: Optional[int] = None):
    n = len(arr) if limit is None else min(limit, len(arr))
    for s in range(0, n, batch_size):
        rows = np.arange(s, min(s + batch_size, n))
        yield valid_candidates(arr, rows, npratio), _pad_history(arr, rows, max_his, truncate)


class DeviceSampler:
    """The shard's impression CSR resident in HBM; each batch is assembled by the
    ``sample_batch`` HIP kernel (no host work, no H2D copy per step).  Same distribution as
    :class:`HostSampler` (a different PRNG: Philox keyed by (seed, rank, step))."""

    def __init__(self, arr: ImpressionArrays, batch_size: int, device, npratio: int = 4, max_his: int = 50,
                 truncate: bool = True, seed: int = 0, rank: int = 0, shuffle: bool = True, drop_last: bool = False):
        import torch

        self.B, self.npratio, self.truncate = batch_size, npratio, truncate
        self.seed, self.rank, self.shuffle, self.drop_last = seed, rank, shuffle, drop_last
        self.n = len(arr)
        lens = np.diff(arr.his_ptr)
        self.H = max_his if truncate else max(max_his, int(lens.max()) if len(lens) else max_his)
        t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt).to(device)
        self.pos = t(arr.pos, torch.int32)
        self.neg_ptr = t(arr.neg_ptr, torch.int64)
        self.negs = t(arr.neg_ids if len(arr.neg_ids) else np.zeros(1, np.int32), torch.int32)
        self.his_ptr = t(arr.his_ptr, torch.int64)
        self.his = t(arr.his_ids if len(arr.his_ids) else np.zeros(1, np.int32), torch.int32)
        self.device = device
        self.step = 0

    def num_batches(self) -> int:
        return self.n // self.B if self.drop_last else -(-self.n // self.B)

    def epoch(self, epoch: int):
        import torch

        from ..ops import native

        lib = native.lib()
        rng = np.random.Generator(np.random.PCG64([self.seed, self.rank, epoch, 17]))
        order = rng.permutation(self.n) if self.shuffle else np.arange(self.n)
        order = torch.as_tensor(order.astype(np.int32)).to(self.device)
        seed = (self.seed * 1_000_003 + self.rank) & 0x7FFFFFFF
        for b in range(self.num_batches()):
            rows = order[b * self.B:(b + 1) * self.B]
            self.step += 1
            yield lib.sample_batch(rows, self.pos, self.neg_ptr, self.negs, self.his_ptr, self.his, self.npratio,
                                   self.H, self.truncate, seed, self.step)

    def valid_batches(self, batch_size: int, limit: Optional[int] = None):
        """The validation batches of :func:`validation_batches` assembled on the device
        (``[pos] + negs[-4:]``, the same history rule), in row order: ``(cand, his)`` device
        tensors, no host work and no H2D copy per batch."""
        import torch

        from ..ops import native

        lib = native.lib()
        n = self.n if limit is None else min(limit, self.n)
        rows = torch.arange(n, dtype=torch.int32, device=self.device)
        for s in range(0, n, batch_size):
            yield lib.sample_batch(rows[s:s + batch_size], self.pos, self.neg_ptr, self.negs, self.his_ptr, self.his,
                                   self.npratio, self.H, self.truncate, 0, 0, True)
