"""Cooperative catalog encode: W client GPUs build the frozen backbone's hidden-state cache
together, each encoding 1/W of the public news catalog.

The reference encodes every title a client touches on that client (``model.py:41-61``
``gen_news_vecs``), and the single-client design here (:class:`..train.news_cache.HiddenCache`)
encodes the client's whole local table once per backbone version.  With W clients on one node
that build is REPLICATED: on synthetic MIND-small at W = 8 every client still holds ~58.5k of the
65k titles and spends ~270 ms encoding them, while its local epoch is only ~294 steps long -- the
build alone amortises to ~0.9 ms per step, twice the step.

The news catalog is public and the frozen backbone's output for a title is the same on every
client (identical weights after the initial sync, deterministic kernels that compute a title's
rows independently of the rest of the batch).  So:

1. **plan** (host, once per run): every client contributes the global ids of its local titles
   over the gloo control group; the union is split so that every title is encoded by exactly
   ONE client that holds its tokens (cyclic preference ``i mod W``, else the next holder), so no
   token table is exchanged and the W shares are balanced;
2. **encode** (device): each client runs the backbone over its share only, in pieces, into a
   send buffer;
3. **gather** (data plane, RCCL over xGMI on the node): one ``all_gather`` per piece -- issued
   asynchronously, so piece ``j`` travels while piece ``j + 1`` is encoded;
4. **place** (device): every client copies the rows of ITS local titles out of the gathered
   catalog into its cache table (one gather launch; the rest is freed).

Nothing about a client's private data leaves it: the exchanged ids are the titles of its local
news table, which (as in the reference's UserData) is the public catalog restricted to the news
its impressions mention -- the data plane moves only backbone outputs of public titles, and every
client receives ALL of them.  A client that needs stronger hiding can pass
``full_news_table=True`` shards (every client then holds the whole catalog).
"""
from __future__ import annotations

import re
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

_NID = re.compile(r"^N(\d+)$")


def global_ids(index2nid: Sequence[str]) -> np.ndarray:
    """Catalog-wide int64 ids of a shard's local rows (``index2nid[row]``): ``N<digits>`` (the
    MIND / synthetic news-id form) -> the number; ``<unk>`` (row 0, the all-zero pad title) ->
    -1; any other string -> a stable 62-bit hash of it (negative, below -1), the same on every
    client."""
    out = np.empty(len(index2nid), dtype=np.int64)
    import hashlib

    for i, n in enumerate(index2nid):
        m = _NID.match(n)
        if m is not None:
            out[i] = int(m.group(1))
        elif n == "<unk>":
            out[i] = -1
        else:
            h = int.from_bytes(hashlib.blake2b(n.encode(), digest_size=8).digest(), "little") >> 2
            out[i] = -2 - h
    return out


@dataclass
class CatalogPlan:
    """Who encodes which catalog title, and where each local row lands after the gather."""

    rank: int
    world: int
    cap: int  # titles per client share (the largest share; the gather's equal block size)
    mine: np.ndarray  # int64 local rows this client encodes, in share order
    src: np.ndarray  # int64 [N_local]: row of the gathered catalog holding local row i
    pieces: int  # all_gather calls (share slots in `pieces` blocks of `piece` titles)
    piece: int
    union: int  # titles in the catalog union
    counts: List[int] = field(default_factory=list)  # share size per client
    plan_s: float = 0.0

    def gathered_row(self, owner: np.ndarray, slot: np.ndarray) -> np.ndarray:
        """Row of the gathered buffer ``[pieces, world, piece]`` for (owner, slot in its share)."""
        return (slot // self.piece) * (self.world * self.piece) + owner * self.piece + slot % self.piece


def _allgather_int64(arr: np.ndarray, group) -> List[np.ndarray]:
    """Variable-length int64 arrays of every member of ``group`` (gloo: host tensors)."""
    W = dist.get_world_size(group)
    n = torch.tensor([arr.size], dtype=torch.int64)
    ns = [torch.zeros(1, dtype=torch.int64) for _ in range(W)]
    dist.all_gather(ns, n, group=group)
    mx = max(int(t.item()) for t in ns)
    buf = torch.full((max(mx, 1),), -(2 ** 62), dtype=torch.int64)
    buf[:arr.size] = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64))
    outs = [torch.empty_like(buf) for _ in range(W)]
    dist.all_gather(outs, buf, group=group)
    return [outs[r][:int(ns[r].item())].numpy() for r in range(W)]


def assign_owners(members: List[np.ndarray]) -> tuple:
    """``members[r]`` = catalog ids client r holds -> ``(union sorted, owner[union])``.

    Title ``i`` of the sorted union prefers client ``i mod W``; when that client does not hold
    it, the next client (cyclically) that does.  Deterministic on every client (same input
    lists), every title owned by exactly one holder, shares balanced to within the overlap
    pattern (W passes of vectorised numpy)."""
    W = len(members)
    union = np.unique(np.concatenate([m for m in members if m.size] or [np.zeros(0, np.int64)]))
    held = np.zeros((W, union.size), dtype=bool)
    for r, m in enumerate(members):
        if m.size:
            held[r, np.searchsorted(union, m)] = True
    owner = np.full(union.size, -1, dtype=np.int64)
    pref = np.arange(union.size) % W
    for k in range(W):
        cand = (pref + k) % W
        take = (owner < 0) & held[cand, np.arange(union.size)]
        owner[take] = cand[take]
    assert (owner >= 0).all(), "a catalog title with no holder"
    return union, owner


def make_plan(local_gids: np.ndarray, rank: int, world: int, ctrl_group, piece_titles: int = 2048) -> CatalogPlan:
    """The cooperative plan of this client (a collective over ``ctrl_group``, gloo, clients
    only).  ``local_gids[i]`` = catalog id of local row ``i`` (:func:`global_ids`; unique)."""
    t0 = time.perf_counter()
    local_gids = np.asarray(local_gids, dtype=np.int64)
    if np.unique(local_gids).size != local_gids.size:
        raise ValueError("cooperative catalog: a client's news table lists a title twice")
    members = _allgather_int64(local_gids, ctrl_group)
    union, owner = assign_owners(members)
    counts = np.bincount(owner, minlength=world)
    cap = int(counts.max()) if counts.size else 0
    # slot of each union title inside its owner's share (share order = union order)
    slot = np.zeros(union.size, dtype=np.int64)
    for r in range(world):
        idx = np.nonzero(owner == r)[0]
        slot[idx] = np.arange(idx.size)
    pieces = max(1, -(-cap // max(1, piece_titles)))
    piece = max(1, -(-cap // pieces))
    # this client's share as local rows
    order = np.argsort(local_gids, kind="stable")
    def local_row(g):  # catalog ids (all held locally) -> local rows
        return order[np.searchsorted(local_gids[order], g)]
    mine_u = np.nonzero(owner == rank)[0]
    mine = local_row(union[mine_u]).astype(np.int64)
    pos = np.searchsorted(union, local_gids)
    plan = CatalogPlan(rank, world, cap, mine, np.zeros(0, np.int64), pieces, piece, int(union.size),
                       [int(c) for c in counts])
    plan.src = plan.gathered_row(owner[pos], slot[pos]).astype(np.int64)
    plan.plan_s = time.perf_counter() - t0
    return plan


def cooperative_build(te, tokens: torch.Tensor, plan: CatalogPlan, data_group, out_dtype: torch.dtype,
                      chunk: int) -> tuple:
    """Encode this client's share, all-gather every share, place the local rows.  Returns
    ``(table [N_local, T, D], timings dict)``; every member of ``data_group`` must call it with
    the same plan geometry (cap / pieces)."""
    dev = tokens.device
    N, _, T = tokens.shape
    D = te.DistillBert.cfg.dim
    W, P, pc = plan.world, plan.pieces, plan.piece
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    t0 = time.perf_counter()
    recv = torch.empty(P, W, pc, T, D, dtype=out_dtype, device=dev)
    send = torch.empty(P, pc, T, D, dtype=out_dtype, device=dev)
    mine = torch.from_numpy(plan.mine).to(dev)
    n_mine = int(plan.mine.size)
    works = []
    t_enc = 0.0
    for p in range(P):
        s0, s1 = p * pc, min((p + 1) * pc, n_mine)
        te0 = time.perf_counter()
        for a in range(s0, s1, chunk):
            b = min(a + chunk, s1)
            rows = tokens.index_select(0, mine[a:b])
            te.hidden(rows, out=send[p, a - s0:b - s0])
        t_enc += time.perf_counter() - te0
        # piece p travels while piece p + 1 is encoded (RCCL: its own stream, ordered after the
        # encode by the collective's stream wait; gloo: a background thread)
        out_list = list(recv[p].unbind(0))
        if dist.get_backend(data_group) == "nccl":
            works.append(dist.all_gather_into_tensor(recv[p], send[p], group=data_group, async_op=True))
        else:
            works.append(dist.all_gather(out_list, send[p], group=data_group, async_op=True))
    for w in works:
        w.wait()
    sync()
    t1 = time.perf_counter()
    del send
    src = torch.from_numpy(plan.src).to(dev)
    table = recv.view(P * W * pc, T, D).index_select(0, src)
    del recv
    sync()
    t2 = time.perf_counter()
    info = {"encode_issue_s": t_enc, "encode_gather_s": t1 - t0, "place_s": t2 - t1, "titles_encoded": n_mine,
            "catalog_titles": plan.union, "share_cap": plan.cap, "pieces": P, "plan_s": plan.plan_s}
    return table, info


def shard_global_ids(shard) -> np.ndarray:
    """:func:`global_ids` of a :class:`..data.shard.Shard` (cached on it)."""
    g = getattr(shard, "_catalog_gids", None)
    if g is None:
        g = global_ids(shard.index2nid)
        shard._catalog_gids = g
    return g


def catalog_owner_counts(plan: CatalogPlan) -> Dict[str, int]:
    return {f"client{r}": c for r, c in enumerate(plan.counts)}


def attach(eng, ctx, piece_titles: int = 2048) -> Optional[CatalogPlan]:
    """Give ``eng`` (a :class:`..train.engine.LocalEngine`) the cooperative plan when EVERY
    client can use it (each has an HBM hidden-state cache -- decided per client by its free
    memory -- and ``FEDREC_COOP_CACHE`` is not 0): one gloo MIN over the clients first, so a
    client without a cache never leaves the others waiting in the gather.  Returns the plan
    (None: every client builds its own table)."""
    import os

    if not ctx.initialized or ctx.num_clients <= 1 or ctx.client_index < 0:
        return None
    ok = eng.hcache is not None and os.environ.get("FEDREC_COOP_CACHE", "1") != "0"
    t = torch.tensor([1 if ok else 0], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.client_ctrl_group)
    if int(t.item()) == 0:
        return None
    plan = make_plan(shard_global_ids(eng.shard), ctx.client_index, ctx.num_clients, ctx.client_ctrl_group,
                     piece_titles)
    eng.set_catalog(plan, ctx.data_group, ctx.client_ctrl_group)
    return plan
