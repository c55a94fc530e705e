"""Reference-format client shard IO plus a compact array form.

On-disk layout (one directory per client, the reference reads ``./UserData``,
``client.py:229-240``):

* ``bert_news_index.npy``  int64 ``[N_news, 2, T]``: WordPiece ids and attention mask;
  row 0 is the all-zero ``<unk>``/pad row (E1).
* ``bert_nid2index.pkl``   ``dict[str -> int]`` (``'<unk>' -> 0``).
* ``train_sam_uid.pkl`` / ``valid_sam_uid.pkl``: ``list`` of
  ``[int, pos_nid, neg_nids, his_nids, uid]`` (unpacked at ``dataset.py:81``).

The pickles are read with :mod:`.safe_pickle` (data opcodes only) and the ``.npy``
with ``allow_pickle=False``.

:class:`Shard` converts the impression lists into CSR int32 arrays, the form the
device sampler (``ops.sample_batch``) consumes: the whole shard lives in HBM and
batches are assembled on the GPU without a host round trip.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import safe_pickle

NEWS_INDEX = "bert_news_index.npy"
NID2INDEX = "bert_nid2index.pkl"
TRAIN_SAM = "train_sam_uid.pkl"
VALID_SAM = "valid_sam_uid.pkl"


@dataclass
class ImpressionArrays:
    """CSR form of a list of ``[_, pos, negs, his, uid]`` rows (ids already mapped)."""

    pos: np.ndarray  # int32 [I]
    neg_ptr: np.ndarray  # int64 [I+1]
    neg_ids: np.ndarray  # int32 [sum negs]
    his_ptr: np.ndarray  # int64 [I+1]
    his_ids: np.ndarray  # int32 [sum his]
    uid: np.ndarray  # int32 [I] (user ordinal within the shard)

    def __len__(self) -> int:
        return int(self.pos.shape[0])

    def negs(self, i: int) -> np.ndarray:
        return self.neg_ids[self.neg_ptr[i]:self.neg_ptr[i + 1]]

    def his(self, i: int) -> np.ndarray:
        return self.his_ids[self.his_ptr[i]:self.his_ptr[i + 1]]

    def subset(self, idx: Sequence[int]) -> "ImpressionArrays":
        idx = np.asarray(idx, dtype=np.int64)
        neg_len = np.diff(self.neg_ptr)[idx]
        his_len = np.diff(self.his_ptr)[idx]
        neg_ptr = np.concatenate([[0], np.cumsum(neg_len)]).astype(np.int64)
        his_ptr = np.concatenate([[0], np.cumsum(his_len)]).astype(np.int64)
        neg_ids = np.concatenate([self.negs(i) for i in idx]) if len(idx) else np.zeros(0, np.int32)
        his_ids = np.concatenate([self.his(i) for i in idx]) if len(idx) else np.zeros(0, np.int32)
        return ImpressionArrays(self.pos[idx].copy(), neg_ptr, neg_ids.astype(np.int32),
                                his_ptr, his_ids.astype(np.int32), self.uid[idx].copy())


def _to_arrays(rows: List[list], nid2index: Dict[str, int]) -> tuple:
    unknown = 0

    def m(n: str) -> int:
        nonlocal unknown
        r = nid2index.get(n)
        if r is None:
            unknown += 1
            return 0
        return r

    uids: Dict[str, int] = {}
    pos, negp, negs, hisp, his, uid = [], [0], [], [0], [], []
    for row in rows:
        _, p, ng, hs, u = row
        pos.append(m(p))
        negs.extend(m(x) for x in ng)
        negp.append(len(negs))
        his.extend(m(x) for x in hs)
        hisp.append(len(his))
        uid.append(uids.setdefault(u, len(uids)))
    arr = ImpressionArrays(
        np.asarray(pos, np.int32), np.asarray(negp, np.int64), np.asarray(negs, np.int32),
        np.asarray(hisp, np.int64), np.asarray(his, np.int32), np.asarray(uid, np.int32))
    return arr, unknown


class Shard:
    """One federated client's private data (reference ``UserData`` directory)."""

    def __init__(self, news_index: np.ndarray, nid2index: Dict[str, int],
                 train: ImpressionArrays, valid: ImpressionArrays, path: Optional[str] = None,
                 index2nid: Optional[List[str]] = None, uids: Optional[List[str]] = None):
        if news_index.ndim != 3 or news_index.shape[1] != 2:
            raise ValueError(f"news index must be [N,2,T], got {news_index.shape}")
        self.news_index = news_index
        self.nid2index = nid2index
        self.train = train
        self.valid = valid
        self.path = path
        self.unknown_train = self.unknown_valid = 0
        self._index2nid = index2nid
        self._uids = uids

    @staticmethod
    def from_lists(news_index: np.ndarray, nid2index: Dict[str, int], train_sam: List[list],
                   valid_sam: List[list], path: Optional[str] = None) -> "Shard":
        train, ut = _to_arrays(train_sam, nid2index)
        valid, uv = _to_arrays(valid_sam, nid2index)
        s = Shard(news_index, nid2index, train, valid, path)
        s.unknown_train, s.unknown_valid = ut, uv
        s._train_sam, s._valid_sam = train_sam, valid_sam
        return s

    # reference list form, materialised lazily (large synthetic shards never need it)
    def _rows(self, arr: ImpressionArrays) -> List[list]:
        i2n = self.index2nid
        uids = self._uids or []
        rows = []
        for i in range(len(arr)):
            u = int(arr.uid[i])
            rows.append([1, i2n[int(arr.pos[i])], [i2n[int(x)] for x in arr.negs(i)],
                         [i2n[int(x)] for x in arr.his(i)], uids[u] if u < len(uids) else f"U{u}"])
        return rows

    @property
    def index2nid(self) -> List[str]:
        if self._index2nid is None:
            inv = ["<unk>"] * self.num_news
            for k, v in self.nid2index.items():
                inv[v] = k
            self._index2nid = inv
        return self._index2nid

    @property
    def train_sam(self) -> List[list]:
        if getattr(self, "_train_sam", None) is None:
            self._train_sam = self._rows(self.train)
        return self._train_sam

    @property
    def valid_sam(self) -> List[list]:
        if getattr(self, "_valid_sam", None) is None:
            self._valid_sam = self._rows(self.valid)
        return self._valid_sam

    # ------------------------------------------------------------------------------
    @property
    def num_news(self) -> int:
        return int(self.news_index.shape[0])

    @property
    def title_len(self) -> int:
        return int(self.news_index.shape[2])

    @staticmethod
    def load(path: str | os.PathLike) -> "Shard":
        p = Path(path)
        news_index = np.load(p / NEWS_INDEX, allow_pickle=False)
        nid2index = safe_pickle.load_path(p / NID2INDEX)
        train_sam = safe_pickle.load_path(p / TRAIN_SAM)
        valid_sam = safe_pickle.load_path(p / VALID_SAM)
        if not isinstance(nid2index, dict) or not isinstance(train_sam, list):
            raise ValueError(f"{p}: unexpected shard object types")
        return Shard.from_lists(news_index, nid2index, train_sam, valid_sam, str(p))

    def save(self, path: str | os.PathLike) -> None:
        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        np.save(p / NEWS_INDEX, self.news_index.astype(np.int64), allow_pickle=False)
        safe_pickle.dump_path(self.nid2index, p / NID2INDEX)
        safe_pickle.dump_path(self.train_sam, p / TRAIN_SAM)
        safe_pickle.dump_path(self.valid_sam, p / VALID_SAM)

    def split_train(self, rank: int, world: int) -> "Shard":
        """Q11 compat: the reference's DistributedSampler re-splits a client's private shard
        by (rank, world) -- ``client.py:249``.  DistributedSampler defaults: shuffle with a
        generator seeded 0 + epoch 0 (``set_epoch`` is never called), pad by repeating the
        head of the permutation, then take ``rank::world``."""
        import torch

        n = len(self.train)
        g = torch.Generator()
        g.manual_seed(0)
        order = torch.randperm(n, generator=g).tolist()
        total = -(-n // world) * world
        pad = total - n
        while pad > 0:
            order += order[:pad]
            pad = total - len(order)
        mine = order[rank:total:world]
        s = Shard.__new__(Shard)
        s.__dict__.update(self.__dict__)
        s._train_sam = None
        s.train = self.train.subset(mine)
        return s
