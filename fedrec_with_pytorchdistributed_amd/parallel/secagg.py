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

Fixed-point arithmetic is what makes cancellation bit-exact.
"""
from __future__ import annotations

import hashlib
import secrets
from typing import List, Optional

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


class RunningMasker:
    """Client ``i``'s secure-aggregation state for repeated sums of one gradient buffer (or
    bucket), with a fixed-point scale that needs no per-step agreement:

    * every coordinate is clamped to a bound ``m`` and quantised on the grid ``2^-f``, ``f``
      the largest with ``W * m * 2^f <= 2^30`` (the W-client int32 sum cannot wrap);
    * ``m`` lives on the device.  It is agreed ONCE, at the first call (the
      scalar MAX all-reduce of ``max|g|``, exact: nothing is clamped), and from then on tracked
      from the PUBLIC result: after each sum every client sets
      ``m = max(headroom * max|sum| / W, decay * m)`` from the
      unmasked sum it holds (``max|sum| / W``: the largest coordinate of the MEAN gradient) -- bitwise identical on every client, so every client derives the
      same ``f`` without a collective, and nothing beyond the sums is disclosed after step 0.
      Clamped coordinates raise the next sum's maximum, so the bound grows back within a
      step; the decay floor keeps it from collapsing on an all-zero step.
    * pair seeds and signs are device-resident (no per-call host->device copy, which torch
      would synchronise on), and the scale is read by the kernels from device memory: a step's
      mask / all-reduce / unmask sequence never waits on the host.

    One SUM all-reduce per call (plus the one-time MAX)."""

    def __init__(self, i: int, world: int, seeds_row: np.ndarray, device: torch.device,
                 headroom: float = 4.0, decay: float = 0.25):
        self.i, self.W, self.row = int(i), int(world), seeds_row
        self.headroom, self.decay = float(headroom), float(decay)
        _, sd, sg = _peer_arrays(self.i, seeds_row)
        self.device = device
        self.sd, self.sg = sd.to(device), sg.to(device)
        self.m: Optional[torch.Tensor] = None  # device fp32 [1]: the current clamp bound

    def _amax(self, g: torch.Tensor) -> torch.Tensor:
        return torch.nan_to_num(g.detach().abs().amax().float().reshape(1), nan=0.0, posinf=3.0e38)

    def allreduce_(self, g: torch.Tensor, round_idx: int, group, check_tag: str = "secagg") -> None:
        """``g`` <- the exact (fixed-point) SUM of every client's ``g``, in place."""
        import torch.distributed as dist

        from .collcheck import CHECK

        if self.m is None:  # one-time agreement of the initial bound
            m = self._amax(g)
            CHECK.record("all_reduce", m, f"{check_tag}-init")
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
            self.m = torch.clamp(m, min=1e-30, max=3.0e38)
        flat = g.reshape(-1)
        if flat.is_cuda:
            from ..ops import native

            lib = native.require_for(flat)
            q = lib.secagg_mask_dev(flat.float().contiguous(), self.sd, self.sg, self.m, self.W, int(round_idx))
            CHECK.record("all_reduce", q, f"{check_tag}-sum")
            dist.all_reduce(q, op=dist.ReduceOp.SUM, group=group)
            lib.secagg_unmask_dev_(q, self.m, self.W, flat)
        else:  # host (gloo plumbing): the same bound rule, the reference-format masks below
            mv = float(self.m.item())
            f = frac_bits_for(self.W, mv)
            q = mask_local(flat, self.i, self.W, self.row, round_idx, f, mv)
            CHECK.record("all_reduce", q, f"{check_tag}-sum")
            dist.all_reduce(q, op=dist.ReduceOp.SUM, group=group)
            flat.copy_(unmask_sum(q, f).view_as(flat))
        self.used = self.m  # the bound this sum was quantised with (tests read it)
        self.m = torch.maximum(torch.clamp(self._amax(flat) * (self.headroom / self.W), max=3.0e38),
                               self.m * self.decay).clamp_(min=1e-30)


def unmask_sum(total: torch.Tensor, frac_bits: int = FRAC_BITS) -> torch.Tensor:
    if total.is_cuda:
        from ..ops import native

        return native.require_for(total).secagg_unmask(total.contiguous(), 2.0 ** -frac_bits)
    return dequantize_ref(total, frac_bits)
