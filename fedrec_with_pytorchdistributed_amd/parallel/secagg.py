"""Secure aggregation by pairwise additive masks (BASELINE config 5).

The reference only *describes* secure aggregation (``README.md:56,65``).  This is the
classic pairwise-masking protocol (Bonawitz et al. 2017, without dropout recovery):

1. **Key agreement** over the control plane: each client draws a secret ``a_i`` and
   publishes ``g^a_i mod p`` (RFC 3526 2048-bit MODP group); every pair derives the same
   seed ``s_ij = SHA-256(g^(a_i a_j) mod p)`` -- the coordinator only ever sees public keys.
2. **Masking** (device kernel ``secagg.hip``): ``y_i = Q(x_i) + sum_{j>i} PRG(s_ij, r) -
   sum_{j<i} PRG(s_ij, r)`` in wrap-around int32 with ``Q(x) = round(clamp(x) * 2^f)``.
3. **Aggregation**: an ordinary int32 SUM all-reduce (RCCL over xGMI); masks cancel
   exactly, leaving ``sum_i Q(x_i)``; then dequantise and divide by ``W``.

Gradient buckets (:class:`ExactMasker`) agree on the fixed-point bound per sum through a
masked exponent histogram, so no value is ever clamped at any number of clients.  The star
mode's model uploads do the same through the store (:class:`StarSecureUpload`): each client
uploads its weighted model DELTA ``(w_k / sum w) (theta_k - theta_global)`` on the grid the
masked histogram agrees, and the coordinator's unmasked sum is the (weighted) FedAvg update to
within ``W 2^(-f-1)`` per coordinate.

Fixed-point arithmetic is what makes cancellation bit-exact.
"""
from __future__ import annotations

import hashlib
import math
import secrets
from typing import List, Optional, Tuple

import numpy as np
import torch

# RFC 3526 group 14 (2048-bit MODP), generator 2
_P = int(
    "FFFFFFFFFFFFFFFFC90FDAA22168C234C4C6628B80DC1CD129024E088A67CC74020BBEA63B139B22514A08798E3404DD"
    "EF9519B3CD3A431B302B0A6DF25F14374FE1356D6D51C245E485B576625E7EC6F44C42E9A637ED6B0BFF5CB6F406B7ED"
    "EE386BFB5A899FA5AE9F24117C4B1FE649286651ECE45B3DC2007CB8A163BF0598DA48361C55D39A69163FA8FD24CF5F"
    "83655D23DCA3AD961C62F356208552BB9ED529077096966D670C354E4ABC9804F1746C08CA18217C32905E462E36CE3B"
    "E39E772C180E86039B2783A2EC07A28FB5C55DF06F4C52C9DE2BCBF6955817183995497CEA956AE515D2261898FA0510"
    "15728E5A8AACAA68FFFFFFFFFFFFFFFF", 16)
_G = 2


class KeyPair:
    def __init__(self, rng_bytes: Optional[bytes] = None):
        raw = rng_bytes if rng_bytes is not None else secrets.token_bytes(32)
        self.secret = int.from_bytes(hashlib.sha256(raw).digest(), "big")
        self.public = pow(_G, self.secret, _P)

    def shared_seed(self, peer_public: int) -> int:
        s = pow(peer_public, self.secret, _P)
        return int.from_bytes(hashlib.sha256(s.to_bytes(256, "big")).digest()[:8], "little") & 0x7FFFFFFFFFFFFFFF


def public_bytes(kp: KeyPair) -> bytes:
    return kp.public.to_bytes(256, "big")


def seeds_from_publics(kp: KeyPair, me: int, publics: List[bytes]) -> np.ndarray:
    """Row ``me`` of the symmetric pair-seed matrix."""
    out = np.zeros(len(publics), dtype=np.int64)
    for j, pb in enumerate(publics):
        if j != me:
            out[j] = kp.shared_seed(int.from_bytes(pb, "big"))
    return out


def pair_seeds(W: int, base_seed: int = 0) -> np.ndarray:
    """Test helper: a full symmetric seed matrix from deterministic key pairs."""
    kps = [KeyPair(f"{base_seed}:{i}".encode()) for i in range(W)]
    pubs = [public_bytes(k) for k in kps]
    return np.stack([seeds_from_publics(kps[i], i, pubs) for i in range(W)])


# ---------------------------------------------------------------------------------------
FRAC_BITS = 16
CLIP = 1024.0


def frac_bits_for(world: int, bound: float) -> int:
    """Fraction bits of the fixed-point grid for ``world`` clients whose coordinates are
    clamped to ``[-bound, bound]``: the largest ``f`` with ``world * bound * 2^f <= 2^30``,
    so the int32 sum of every client's quantised value cannot wrap (masks aside).  The same
    rule as the device kernels' ``frac_exp2`` (``secagg.hip``)."""
    import math

    f = int(math.floor(math.log2((2.0 ** 30) / (max(1, int(world)) * max(float(bound), 1e-30)))))
    return max(0, min(f, 56))


def quantize_ref(x: torch.Tensor, frac_bits: int = FRAC_BITS, clip: float = CLIP) -> torch.Tensor:
    return torch.round(x.float().clamp(-clip, clip) * (2.0 ** frac_bits)).to(torch.int64).to(torch.int32)


def dequantize_ref(q: torch.Tensor, frac_bits: int = FRAC_BITS) -> torch.Tensor:
    return q.float() * (2.0 ** -frac_bits)


def _peer_arrays(i: int, seeds_row: np.ndarray):
    peers = [j for j in range(len(seeds_row)) if j != i]
    sd = torch.tensor([int(seeds_row[j]) for j in peers], dtype=torch.int64)
    sg = torch.tensor([1 if i < j else -1 for j in peers], dtype=torch.int32)
    return peers, sd, sg


def mask_local(x: torch.Tensor, i: int, W: int, seeds: np.ndarray, round_idx: int,
               frac_bits: int = FRAC_BITS, clip: float = CLIP) -> torch.Tensor:
    """Client ``i``'s masked fixed-point upload (int32, wrap-around)."""
    row = seeds[i] if seeds.ndim == 2 else seeds
    peers, sd, sg = _peer_arrays(i, row)
    flat = x.reshape(-1).float().contiguous()
    if flat.is_cuda:
        from ..ops import native

        out = native.require_for(flat).secagg_mask(flat, sd, sg, float(2.0 ** frac_bits), float(clip), int(round_idx))
        if isinstance(out, (tuple, list)):
            out = out[0]
        return out.view(x.shape)
    q = quantize_ref(flat, frac_bits, clip).numpy().astype(np.uint32)
    acc = q.copy()
    for s, g in zip(sd.tolist(), sg.tolist()):
        r = np.random.Generator(np.random.PCG64([s & 0xFFFFFFFFFFFFFFFF, round_idx])).integers(
            0, 1 << 32, flat.numel(), dtype=np.uint64).astype(np.uint32)
        acc = (acc + r) if g > 0 else (acc - r)  # uint32 wrap-around
    return torch.from_numpy(acc.view(np.int32).copy()).view(x.shape)


HIST_SLOTS = 256
_HIST_ROUND = 1 << 62  # PRG counter space of the exponent histograms (disjoint from the payloads')


def hist_slot(max_abs: float) -> int:
    """Histogram slot of a client's largest finite ``|x|`` (the device kernels' rule): 0 for 0,
    else ``max(e, 1) + 1`` with ``e`` the fp32 exponent field, so slot ``s`` means
    ``max|x| < 2^(s - 127)``."""
    bits = int(np.array([max_abs], dtype=np.float32).view(np.uint32)[0])
    if bits == 0:
        return 0
    return max(bits >> 23, 1) + 1


def hist_local(x: torch.Tensor) -> np.ndarray:
    """This client's UNMASKED histogram: a one-hot at :func:`hist_slot` of its max|x| and, in
    slot 1, its count of non-finite coordinates."""
    v = x.detach().reshape(-1).float().abs()
    fin = torch.isfinite(v)
    h = np.zeros(HIST_SLOTS, dtype=np.int64)
    h[hist_slot(float(v[fin].max()) if bool(fin.any()) else 0.0)] += 1
    h[1] += int((~fin).sum())
    return h


def hist_frac_bits(H, world: int) -> Tuple[int, bool]:
    """``(f, non_finite)`` from a SUMMED histogram: the bound is ``2^E`` of the largest occupied
    slot and ``f = 30 - ceil(log2 W) - E`` (clamped to [-120, 60]) -- the W-client int32 sum of
    values within the bound cannot wrap, and no client's value exceeds it."""
    H = np.asarray(H).reshape(-1)
    occ = [s for s in range(2, HIST_SLOTS) if H[s] != 0]
    bad = bool(H[1] != 0)
    if not occ:
        return 0, bad
    E = max(occ) - 127
    f = 30 - int(math.ceil(math.log2(max(1, int(world))))) - E
    return max(-120, min(60, f)), bad


def _add_masks(acc: np.ndarray, seeds_row: np.ndarray, i: int, round_idx: int) -> np.ndarray:
    """uint32 wrap-around ``acc + sum_j sign_ij PRG(s_ij, round)`` (host PRG: PCG64)."""
    peers, sd, sg = _peer_arrays(i, seeds_row)
    for s, g in zip(sd.tolist(), sg.tolist()):
        r = np.random.Generator(np.random.PCG64([s & 0xFFFFFFFFFFFFFFFF, round_idx])).integers(
            0, 1 << 32, acc.size, dtype=np.uint64).astype(np.uint32)
        acc = (acc + r) if g > 0 else (acc - r)
    return acc


class ExactMasker:
    """Client ``i``'s end of an EXACT secure sum of a gradient buffer (or bucket), any number
    of clients, no host synchronisation on the device:

    1. **bound agreement** -- a masked exponent histogram (:data:`HIST_SLOTS` int32): each
       client adds a one-hot at the binary exponent of its own ``max|g|`` (and its count of
       non-finite coordinates); one SUM all-reduce of 1 KB; every client reads the largest
       occupied slot, a power of two ``m >= max_k max|g_k|``.  The masks hide which client
       holds which exponent: the sum discloses only how many clients have their maximum in
       each power-of-two range.
    2. **payload** -- ``Q(g) = round(g 2^f)`` with ``f = 30 - ceil(log2 W) - log2 m`` (the
       W-client sum cannot wrap int32), pairwise masks, one int32 SUM all-reduce; the masks
       cancel exactly and the dequantised sum is the plain sum to within ``W 2^(-f-1)``.

    Nothing is clamped, so there is no running bound to collapse or to lag a gradient spike
    (round 3's ``RunningMasker``).  A non-finite coordinate anywhere makes every output NaN,
    as the plain sum would be non-finite.  Two collectives per call, both on the caller's
    stream."""

    def __init__(self, i: int, world: int, seeds_row: np.ndarray, device: torch.device):
        self.i, self.W, self.row = int(i), int(world), seeds_row
        _, sd, sg = _peer_arrays(self.i, seeds_row)
        self.device = device
        self.sd, self.sg = sd.to(device), sg.to(device)
        self.hist: Optional[torch.Tensor] = None  # the last summed histogram (tests read it)

    def frac_bits(self) -> int:
        """Fraction bits of the last sum (reads the device histogram: tests / diagnostics)."""
        return hist_frac_bits(self.hist.cpu().numpy(), self.W)[0]

    def allreduce_(self, g: torch.Tensor, round_idx: int, group, check_tag: str = "secagg", ipc=None) -> None:
        """``g`` <- the exact (fixed-point) SUM of every client's ``g``, in place.  ``ipc``: an
        :class:`.ipc_allreduce.IpcAllReduce` moves both int32 buffers instead of ``group``."""
        import torch.distributed as dist

        from .collcheck import CHECK

        flat = g.reshape(-1)
        hround = _HIST_ROUND | int(round_idx)
        if flat.is_cuda:
            from ..ops import native

            lib = native.require_for(flat)
            x = flat if (flat.dtype == torch.float32 and flat.is_contiguous()) else flat.float().contiguous()
            h = lib.secagg_hist(x, self.sd, self.sg, hround)
            CHECK.record("all_reduce", h, f"{check_tag}-hist")
            if ipc is not None:
                ipc.allreduce_(h)
            else:
                dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            q = lib.secagg_mask_exact(x, self.sd, self.sg, h, self.W, int(round_idx))
            CHECK.record("all_reduce", q, f"{check_tag}-sum")
            if ipc is not None:
                ipc.allreduce_(q)
            else:
                dist.all_reduce(q, op=dist.ReduceOp.SUM, group=group)
            if x is flat:
                lib.secagg_unmask_exact_(q, h, self.W, flat)
            else:
                out = torch.empty_like(x)
                lib.secagg_unmask_exact_(q, h, self.W, out)
                flat.copy_(out)
            self.hist = h
            return
        # host (gloo plumbing): the same protocol with the host PRG
        hl = _add_masks(hist_local(flat).astype(np.uint32), self.row, self.i, hround)
        h = torch.from_numpy(hl.view(np.int32).copy())
        CHECK.record("all_reduce", h, f"{check_tag}-hist")
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        f, bad = hist_frac_bits(h.numpy(), self.W)
        v = flat.detach().float()
        v = torch.where(torch.isfinite(v), v, torch.zeros_like(v))
        qv = torch.round(v.double() * (2.0 ** f)).to(torch.int64).numpy().astype(np.uint32)
        q = torch.from_numpy(_add_masks(qv, self.row, self.i, int(round_idx)).view(np.int32).copy())
        CHECK.record("all_reduce", q, f"{check_tag}-sum")
        dist.all_reduce(q, op=dist.ReduceOp.SUM, group=group)
        out = q.double() * (2.0 ** -f)
        if bad:
            out.fill_(float("nan"))
        flat.copy_(out.to(flat.dtype).view_as(flat))
        self.hist = h


def masked_hist_host(x: torch.Tensor, i: int, seeds_row: np.ndarray, round_idx: int) -> torch.Tensor:
    """Client ``i``'s masked exponent histogram of ``x`` (:func:`hist_local` + the pairwise
    masks of counter ``_HIST_ROUND | round_idx``), int32 [HIST_SLOTS] on the host."""
    h = _add_masks(hist_local(x).astype(np.uint32), seeds_row, i, _HIST_ROUND | int(round_idx))
    return torch.from_numpy(h.view(np.int32).copy())


def sum_wrap(ts: List[torch.Tensor]) -> torch.Tensor:
    """uint32 wrap-around sum of int32 tensors (the masks cancel in it), on the host."""
    acc = ts[0].reshape(-1).numpy().astype(np.uint32).copy()
    for t in ts[1:]:
        acc += t.reshape(-1).numpy().astype(np.uint32)
    return torch.from_numpy(acc.view(np.int32).copy()).view(ts[0].shape)


class StarSecureUpload:
    """The star (FedAvg) mode's exact secure upload, over the store control plane.

    Round ``r``, client ``k`` with the round's global model ``theta_g`` and its trained
    ``theta_k``:

    1. weights: ``w_k`` (1, or the sample count under ``weighted_fedavg``) is published --
       the coordinator already receives it in the round's metadata -- and every client reads
       ``sum w``;
    2. ``u_k = (w_k / sum w) (theta_k - theta_g)``: the weight is applied BEFORE quantising and
       the delta (a few Adam steps) is what goes on the grid, not the parameters;
    3. bound agreement: the masked exponent histogram of ``u_k`` goes to the store; every
       client (and the coordinator) sums the W blobs, the masks cancel, and the largest
       occupied slot gives ``m = 2^E >= max_k max|u_k|`` and ``f = 30 - ceil(log2 W) - E``;
    4. payload: ``round(u_k 2^f)`` (nothing clamped: ``|u_k| <= m``) + pairwise masks.

    The coordinator's wrap-around sum of the W payloads unmasks to ``sum_k u_k`` within
    ``W 2^(-f-1)``; the new global model is ``theta_g + sum_k u_k`` = the (weighted) mean of
    the ``theta_k``, as ``server.py:46-50`` computes it in the clear.  Disclosed beyond the
    sum: the weights (already in the metadata) and how many clients have their largest
    ``|u_k|`` in each power-of-two range (the summed histogram)."""

    def __init__(self, cp, k: int, world: int, seeds_row: np.ndarray):
        self.cp, self.k, self.W, self.row = cp, int(k), int(world), seeds_row

    def upload(self, r: int, theta_k: torch.Tensor, theta_g: torch.Tensor, weight: float) -> dict:
        cp, k, W = self.cp, self.k, self.W
        cp.put_json(f"r{r}/w/{k}", {"w": float(weight)})
        ws = [float(cp.get_json(f"r{r}/w/{j}")["w"]) for j in range(W)]
        u = (theta_k.float() - theta_g.float()) * float(weight / sum(ws))
        cp.put_tensor(f"r{r}/hist/{k}", masked_hist_host(u, k, self.row, r))
        H = sum_wrap([cp.get_tensor(f"r{r}/hist/{j}") for j in range(W)])
        f, bad = hist_frac_bits(H.numpy(), W)
        occ = [s for s in range(2, HIST_SLOTS) if int(H[s]) != 0]
        bound = 2.0 ** (max(occ) - 127) if occ else 1.0
        if bad:  # a non-finite coordinate somewhere: upload zeros; the coordinator rejects the round
            u = torch.zeros_like(u)
        masked = mask_local(u, k, W, self.row, r, f, bound)
        cp.put_tensor(f"r{r}/up/{k}", masked.cpu())
        return {"frac_bits": f, "non_finite": bad, "sum_w": sum(ws)}


def star_secure_aggregate(cp, r: int, world: int, ups: List[torch.Tensor], theta_g: torch.Tensor):
    """Coordinator side of :class:`StarSecureUpload`: ``(new global, frac_bits)`` from the W
    masked uploads of round ``r`` (None when a client reported a non-finite coordinate)."""
    H = sum_wrap([cp.get_tensor(f"r{r}/hist/{j}") for j in range(world)])
    f, bad = hist_frac_bits(H.numpy(), world)
    if bad:
        return None, f
    tot = sum_wrap([u.cpu() for u in ups])
    upd = tot.double() * (2.0 ** -f)
    return (theta_g.double().cpu() + upd.view(theta_g.shape)).float(), f


def unmask_sum(total: torch.Tensor, frac_bits: int = FRAC_BITS) -> torch.Tensor:
    if total.is_cuda:
        from ..ops import native

        return native.require_for(total).secagg_unmask(total.contiguous(), 2.0 ** -frac_bits)
    return dequantize_ref(total, frac_bits)
