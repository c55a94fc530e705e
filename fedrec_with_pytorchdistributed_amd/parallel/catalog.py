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

Agreement checks (a cooperative table must equal the one each client would build alone):
the clients' frozen backbones are compared by an exact integer digest of every weight
(:func:`backbone_digest`), and the token rows of every shared title by a 64-bit hash
(:func:`token_row_hashes`) -- a client whose backbone or tokenisation differs would otherwise
receive another client's hidden states for its rows.  Any disagreement makes every client fall
back to its own local build (with a log line); the decision is taken on gathered data, so all
clients take it together.

Memory: the gathered pieces are placed into the table as they arrive (a ring of two receive
pieces), so the build's transient peak is the table + two pieces, not the whole union; that peak
is checked against every client's free memory before the plan is accepted.

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

_NID = re.compile(r"^N([1-9]\d*|0)$")  # canonical numbers only: 'N0123' must not alias 'N123'



class CatalogMismatch(RuntimeError):
    """The clients disagree on what a shared title (its tokens) or the backbone is."""


_MIX = 0x9E3779B97F4A7C15 - (1 << 64)  # odd 64-bit constant as a signed int64


@torch.no_grad()
def token_row_hashes(tokens: torch.Tensor) -> np.ndarray:
    """A 64-bit polynomial hash of every title's token row (``tokens [N, 2, T]``: ids + mask),
    computed where the table lives (int64 arithmetic wraps mod 2^64: exact, order-free)."""
    n = tokens.shape[0]
    x = tokens.reshape(n, -1).to(torch.int64) + 1
    L = x.shape[1]
    coef = (torch.arange(1, L + 1, dtype=torch.int64, device=x.device) * _MIX) | 1
    return ((x * coef).sum(dim=1) * _MIX).cpu().numpy()


@torch.no_grad()
def backbone_digest(backbone) -> int:
    """Exact digest of every weight's BITS (a position-weighted int64 sum per tensor, folded in
    order): clients agree iff their frozen backbones are bitwise identical (up to 2^-64)."""
    h = 0
    for p in backbone.parameters():
        x = p.detach().contiguous().view(-1)
        xi = {8: torch.int64, 4: torch.int32, 2: torch.int16, 1: torch.int8}[x.element_size()]
        xi = x.view(xi).to(torch.int64)
        w = (torch.arange(1, xi.numel() + 1, dtype=torch.int64, device=x.device) * _MIX) | 1
        v = int((xi * w).sum().item())
        h = ((h * 1000003) ^ (v & ((1 << 64) - 1))) & ((1 << 63) - 1)
    return h


def global_ids(index2nid: Sequence[str]) -> np.ndarray:
    """Catalog-wide int64 ids of a shard's local rows (``index2nid[row]``): ``N<digits>`` (the
    MIND / synthetic news-id form, no leading zero) -> the number; ``<unk>`` (row 0, the
    all-zero pad title) -> -1; any other string (``N0123`` included) -> a stable 62-bit hash of it
    (negative, below -1), the same on every client."""
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


def _check_token_hashes(members: List[np.ndarray], hashes: List[np.ndarray]) -> None:
    """Every holder of a catalog id must hold the same token row (else :class:`CatalogMismatch`)."""
    gid = np.concatenate([m for m in members] or [np.zeros(0, np.int64)])
    hh = np.concatenate([h for h in hashes] or [np.zeros(0, np.int64)])
    if gid.size == 0:
        return
    order = np.lexsort((hh, gid))
    g, h = gid[order], hh[order]
    same_id = g[1:] == g[:-1]
    bad = same_id & (h[1:] != h[:-1])
    if bad.any():
        i = int(np.nonzero(bad)[0][0])
        raise CatalogMismatch(f"cooperative catalog: {int(bad.sum())} shared title id(s) carry different token "
                              f"rows on different clients (first: catalog id {int(g[i])})")


def make_plan(local_gids: np.ndarray, rank: int, world: int, ctrl_group, piece_titles: int = 2048,
              token_hashes: Optional[np.ndarray] = None) -> CatalogPlan:
    """The cooperative plan of this client (a collective over ``ctrl_group``, gloo, clients
    only).  ``local_gids[i]`` = catalog id of local row ``i`` (:func:`global_ids`; unique).
    ``token_hashes[i]`` (:func:`token_row_hashes`): checked equal across the holders of every
    shared id -- raises :class:`CatalogMismatch` on every client alike (gathered data)."""
    t0 = time.perf_counter()
    local_gids = np.asarray(local_gids, dtype=np.int64)
    if np.unique(local_gids).size != local_gids.size:
        raise ValueError("cooperative catalog: a client's news table lists a title twice")
    members = _allgather_int64(local_gids, ctrl_group)
    if token_hashes is not None:
        th = np.asarray(token_hashes, dtype=np.int64)
        if th.shape != local_gids.shape:
            raise ValueError("cooperative catalog: one token hash per local title")
        _check_token_hashes(members, _allgather_int64(th, ctrl_group))
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


def transient_bytes(plan: CatalogPlan, title_len: int, dim: int, elem: int) -> int:
    """Device bytes a cooperative build holds besides the table: a ring of two receive pieces
    ([W, piece] titles each) and two send pieces, plus one piece of placed rows in flight."""
    row = title_len * dim * elem
    return row * plan.piece * (2 * plan.world + 2 + plan.world)


RING = 2  # receive / send pieces alive at once (piece p travels while p + 1 is encoded)


def cooperative_build(te, tokens: torch.Tensor, plan: CatalogPlan, data_group, out_dtype: torch.dtype,
                      chunk: int) -> tuple:
    """Encode this client's share, all-gather every share, place the local rows.  Returns
    ``(table [N_local, T, D], timings dict)``; every member of ``data_group`` must call it with
    the same plan geometry (cap / pieces).  Pieces are placed as they land: only RING receive
    pieces exist at a time (the whole union is never held)."""
    dev = tokens.device
    N, _, T = tokens.shape
    D = te.DistillBert.cfg.dim
    W, P, pc = plan.world, plan.pieces, plan.piece
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    t0 = time.perf_counter()
    table = torch.empty(N, T, D, dtype=out_dtype, device=dev)
    nr = min(RING, P)
    recv = [torch.empty(W * pc, T, D, dtype=out_dtype, device=dev) for _ in range(nr)]
    send = [torch.empty(pc, T, D, dtype=out_dtype, device=dev) for _ in range(nr)]
    mine = torch.from_numpy(plan.mine).to(dev)
    n_mine = int(plan.mine.size)
    # local rows whose source row lies in piece p, and that row's index inside the piece
    piece_of = plan.src // (W * pc)
    place_idx = []
    for p in range(P):
        loc = np.nonzero(piece_of == p)[0]
        place_idx.append((torch.from_numpy(loc.astype(np.int64)).to(dev),
                          torch.from_numpy((plan.src[loc] - p * W * pc).astype(np.int64)).to(dev)))
    nccl = dist.get_backend(data_group) == "nccl"
    works: List = [None] * P
    t_enc = t_place = 0.0

    def place(p: int) -> None:
        nonlocal t_place
        works[p].wait()  # (RCCL: the current stream waits for the gather)
        tp = time.perf_counter()
        loc, row = place_idx[p]
        if loc.numel():
            table.index_copy_(0, loc, recv[p % nr].index_select(0, row))
        t_place += time.perf_counter() - tp

    for p in range(P):
        b = p % nr
        if p >= nr:
            place(p - nr)  # frees receive + send buffer b (the gather that read send[b] is done)
        s0, s1 = p * pc, min((p + 1) * pc, n_mine)
        te0 = time.perf_counter()
        for a in range(s0, s1, chunk):
            e = min(a + chunk, s1)
            rows = tokens.index_select(0, mine[a:e])
            te.hidden(rows, out=send[b][a - s0:e - s0])
        t_enc += time.perf_counter() - te0
        # piece p travels while piece p + 1 is encoded (RCCL: its own stream, ordered after the
        # encode by the collective's stream wait; gloo: a background thread)
        if nccl:
            works[p] = dist.all_gather_into_tensor(recv[b], send[b], group=data_group, async_op=True)
        else:
            works[p] = dist.all_gather(list(recv[b].view(W, pc, T, D).unbind(0)), send[b], group=data_group,
                                       async_op=True)
    for p in range(max(0, P - nr), P):
        place(p)
    sync()
    t1 = time.perf_counter()
    del send, recv
    info = {"encode_issue_s": t_enc, "encode_gather_s": t1 - t0, "place_s": t_place, "titles_encoded": n_mine,
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


def attach(eng, ctx, piece_titles: int = 2048, log=None) -> Optional[CatalogPlan]:
    """Give ``eng`` (a :class:`..train.engine.LocalEngine`) the cooperative plan when EVERY
    client can use it: each has an HBM hidden-state cache (decided per client by its free
    memory) and ``FEDREC_COOP_CACHE`` is not 0 (one gloo MIN first, so a client without a cache
    never leaves the others waiting in the gather); the frozen backbones are bitwise identical
    (:func:`backbone_digest`, all-gathered); every shared title has the same token row on every
    holder (:func:`token_row_hashes`, checked in :func:`make_plan`); and the build's transient
    peak (:func:`transient_bytes`) fits every client's free memory beside its table.  Returns the
    plan, or None: every client builds its own table (a log line says why)."""
    import os

    from ..utils import obs

    say = log or obs.log
    if not ctx.initialized or ctx.num_clients <= 1 or ctx.client_index < 0:
        return None
    ok = eng.hcache is not None and os.environ.get("FEDREC_COOP_CACHE", "1") != "0"
    t = torch.tensor([1 if ok else 0], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.client_ctrl_group)
    if int(t.item()) == 0:
        return None
    W = ctx.num_clients
    mine = torch.tensor([backbone_digest(eng.model.text_encoder.DistillBert)], dtype=torch.int64)
    digs = [torch.zeros(1, dtype=torch.int64) for _ in range(W)]
    dist.all_gather(digs, mine, group=ctx.client_ctrl_group)
    if len({int(d.item()) for d in digs}) > 1:
        eng.catalog_refused = "backbone weights differ across clients"
        say(f"[client {ctx.client_index}] cooperative catalog off: the clients' frozen backbones differ "
            f"(digests {[hex(int(d.item()))[:12] for d in digs]}); every client builds its own cache")
        return None
    try:
        plan = make_plan(shard_global_ids(eng.shard), ctx.client_index, W, ctx.client_ctrl_group, piece_titles,
                         token_hashes=token_row_hashes(eng.tokens))
    except CatalogMismatch as e:
        eng.catalog_refused = str(e)
        say(f"[client {ctx.client_index}] cooperative catalog off: {e}; every client builds its own cache")
        return None
    # the build's peak beside the table must fit this client's device memory (agreed by MIN)
    fits = 1
    dev = eng.device
    if dev.type == "cuda":
        te = eng.model.text_encoder
        T = int(eng.tokens.shape[2])
        elem = torch.empty((), dtype=te.compute_dtype).element_size()
        need = eng.N * T * te.DistillBert.cfg.dim * elem + transient_bytes(plan, T, te.DistillBert.cfg.dim, elem)
        free, _ = torch.cuda.mem_get_info(dev)
        # the local build's rule (table <= free / 4) leaves the backbone's chunk activations
        # room; the cooperative peak gets the same headroom: table + transient <= free / 2
        fits = int(need <= free // 2)
        if not fits:
            say(f"[client {ctx.client_index}] cooperative catalog: peak {need / 2**30:.1f} GiB > half of "
                f"{free / 2**30:.1f} GiB free")
    t = torch.tensor([fits], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.client_ctrl_group)
    if int(t.item()) == 0:
        eng.catalog_refused = "the cooperative build's peak memory does not fit every client"
        return None
    eng.set_catalog(plan, ctx.data_group, ctx.client_ctrl_group)
    return plan
