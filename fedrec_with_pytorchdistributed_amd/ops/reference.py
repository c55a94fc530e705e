"""Torch-eager oracle for every fused op (fp32).  This is both the CPU execution path
(BASELINE config 1: CPU/gloo plumbing) and the numerics reference that each HIP kernel is
tested against.

Math is traced to the reference:

* DistilBERT block: HF post-LN block; attention scores ``q k^T / sqrt(d)`` with key padding
  filled with ``finfo.min`` (so an all-zero mask -- news row 0 -- gives a *uniform*
  softmax, E1/K03), GELU(erf) FFN, LayerNorm eps 1e-12.
* Additive attention (``attention.py:14-26``): ``alpha = exp(a) / (sum exp(a) + 1e-8)``
  with ``a = w2 . tanh(W1 x + b1) + b2``; no mask (Q7).
* Scaled dot-product attention (``attention.py:37-45``): ``A = exp(S) / (rowsum + 1e-8)``,
  no max subtraction (Q8), no mask.
* Score (``model.py:121-126``): ``CE(sigmoid(<cand, u>), label=0)``, mean over the batch.

The eps-normalised softmaxes are evaluated in the algebraically identical stable form
``exp(s - m) / (sum exp(s - m) + eps * exp(-m))`` (identical in exact arithmetic; the
literal form overflows for scores > 88).  ``literal=True`` selects the reference's form.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

EPS_SOFTMAX = 1e-8


def _f(t: torch.Tensor) -> torch.Tensor:
    """Compute dtype of the oracle: fp32, or fp64 when the caller is in fp64 (tests)."""
    return t if t.dtype == torch.float64 else t.float()


# ---------------------------------------------------------------------------------------
# eps-softmax helpers
# ---------------------------------------------------------------------------------------
def eps_softmax(s: torch.Tensor, dim: int, eps: float = EPS_SOFTMAX, literal: bool = False,
                keep: torch.Tensor | None = None) -> torch.Tensor:
    """``exp(s) / (sum exp(s) + eps)`` in the stable form.  ``keep`` (bool, broadcastable to
    ``s``): masked entries get weight exactly 0; a slice with every entry masked is all 0
    (max taken as 0) -- the kernels' mask_padding semantics."""
    if keep is not None:
        s = s.masked_fill(~keep, float("-inf"))
        m = s.amax(dim, keepdim=True)
        m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
        e = torch.exp(s - m)
        return e / (e.sum(dim, keepdim=True) + eps * torch.exp(-m))
    if literal:
        e = torch.exp(s)
        return e / (e.sum(dim, keepdim=True) + eps)
    m = s.amax(dim, keepdim=True).clamp_min(-1e30)
    e = torch.exp(s - m)
    return e / (e.sum(dim, keepdim=True) + eps * torch.exp(-m))


def eps_softmax_backward(p: torch.Tensor, dp: torch.Tensor, dim: int) -> torch.Tensor:
    """``d s`` for ``p = eps_softmax(s)``: the eps term only rescales, so the Jacobian keeps
    the softmax form ``p (dp - sum p dp)``."""
    return p * (dp - (p * dp).sum(dim, keepdim=True))


# ---------------------------------------------------------------------------------------
# counter-based RNG (bit-exact twin of csrc/common.h Philox / drop_scale)
# ---------------------------------------------------------------------------------------
_U32 = 0xFFFFFFFF


def philox4x32(seed: int, offset: int, ctr: torch.Tensor) -> torch.Tensor:
    """Philox-4x32-10 (Salmon et al. 2011) with the kernels' layout: counter words
    (ctr lo, ctr hi, offset lo, offset hi), key (seed lo, seed hi).  ``ctr`` int64 -> ``[..., 4]``
    int64 holding uint32 values.  int64 products wrap mod 2^64, which keeps the low 64 bits of
    the 32x32 product exact -- all mul-hi / mul-lo need."""
    ctr = ctr.to(torch.int64)
    c0, c1 = ctr & _U32, (ctr >> 32) & _U32
    c2 = torch.full_like(ctr, int(offset) & _U32)
    c3 = torch.full_like(ctr, (int(offset) >> 32) & _U32)
    k0, k1 = int(seed) & _U32, (int(seed) >> 32) & _U32
    for _ in range(10):
        p0 = c0 * 0xD2511F53
        p1 = c2 * 0xCD9E8D57
        c0, c1, c2, c3 = ((p1 >> 32) & _U32) ^ c1 ^ k0, p1 & _U32, ((p0 >> 32) & _U32) ^ c3 ^ k1, p0 & _U32
        k0 = (k0 + 0x9E3779B9) & _U32
        k1 = (k1 + 0xBB67AE85) & _U32
    return torch.stack([c0, c1, c2, c3], -1)


def _keep_scale(words: torch.Tensor, p: float) -> torch.Tensor:
    """uint32 words (int64) -> dropout multipliers: keep / (1 - p), keep iff unit(x) > p."""
    u = ((words >> 8) + 1).to(torch.float32) * (1.0 / 16777216.0)
    pf = torch.tensor(p, dtype=torch.float32)
    inv_keep = torch.tensor(1.0, dtype=torch.float32) / (1.0 - pf)
    return torch.where(u > pf, inv_keep, torch.zeros((), dtype=torch.float32))


def dropout_scale(index: torch.Tensor, p: float, seed: int, offset: int) -> torch.Tensor:
    """Dropout multiplier of element ``index`` (int64): ``keep / (1 - p)`` with keep iff
    ``unit(x) > p`` where x = component ``index & 3`` of Philox counter ``index >> 2``."""
    x = philox4x32(seed, offset, index >> 2).gather(-1, (index & 3).unsqueeze(-1)).squeeze(-1)
    return _keep_scale(x, p)


def dropout_add(h: torch.Tensor, res: Optional[torch.Tensor], p: float, seed: int, offset: int) -> torch.Tensor:
    """``res + h o Z`` with Z the element-indexed mask of ``csrc/dropout.hip`` (one Philox
    call per 4 consecutive elements, as the kernel)."""
    n = h.numel()
    words = philox4x32(seed, offset, torch.arange((n + 3) // 4, device=h.device)).reshape(-1)[:n]
    z = _keep_scale(words, p).view(h.shape).to(_f(h).dtype)
    out = _f(h) * z
    return out if res is None else out + _f(res)


def attention_dropout_scale(n: int, n_heads: int, T: int, p: float, seed: int, offset: int) -> torch.Tensor:
    """``[n, h, T, T]`` multipliers of the attention probabilities: element (title, head, t, s)
    is mask index ``((title * h + head) * 64 + t) * 64 + s`` (title_attn.hip, T <= 64), i.e.
    Philox counter ``(pair * 64 + t) * 16 + s // 4``, word ``s % 4``."""
    g = (T + 3) // 4
    pair = torch.arange(n * n_heads, dtype=torch.int64).view(-1, 1, 1)
    t = torch.arange(T, dtype=torch.int64).view(1, T, 1)
    q = torch.arange(g, dtype=torch.int64).view(1, 1, g)
    words = philox4x32(seed, offset, (pair * 64 + t) * 16 + q).reshape(n * n_heads, T, 4 * g)[..., :T]
    return _keep_scale(words, p).view(n, n_heads, T, T)


# ---------------------------------------------------------------------------------------
# text backbone (DistilBERT-shaped) pieces
# ---------------------------------------------------------------------------------------
def embed_ln(tokens: torch.Tensor, word: torch.Tensor, pos: torch.Tensor, ln_w: torch.Tensor,
             ln_b: torch.Tensor, eps: float) -> torch.Tensor:
    """``LN(word[tok] + pos[0..T-1])`` -> ``[n*T, D]`` (HF Embeddings, eval mode)."""
    n, T = tokens.shape
    # F.embedding(padding_idx=0) like HF's nn.Embedding: the pad row gets no gradient
    x = F.embedding(tokens.long(), word, padding_idx=0) + pos[:T].unsqueeze(0)
    x = F.layer_norm(_f(x), (word.shape[1],), _f(ln_w), _f(ln_b), eps)
    return x.reshape(n * T, -1)


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], act: str = "none",
           residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    y = _f(x) @ _f(w).t()
    if b is not None:
        y = y + _f(b)
    if act == "gelu":
        y = F.gelu(y)  # erf form (HF "gelu")
    elif act == "tanh":
        y = torch.tanh(y)
    elif act != "none":
        raise ValueError(act)
    if residual is not None:
        y = y + _f(residual)
    return y


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    return F.layer_norm(_f(x), (x.shape[-1],), _f(w), _f(b), eps)


def title_attention(qkv: torch.Tensor, mask: torch.Tensor, n_heads: int, drop=None) -> torch.Tensor:
    """HF DistilBERT eager attention.  ``qkv`` ``[n*T, 3D]`` (q | k | v), ``mask`` ``[n, T]``;
    ``drop = (p, seed, offset)``: train-mode dropout on the probabilities (HF
    ``nn.functional.dropout(attn_weights)``) with the kernels' Philox mask."""
    n, T = mask.shape
    D = qkv.shape[1] // 3
    dh = D // n_heads
    q, k, v = _f(qkv).view(n, T, 3, n_heads, dh).permute(2, 0, 3, 1, 4)
    q = q / math.sqrt(dh)
    s = q @ k.transpose(-1, -2)  # [n, h, T, T]
    keep = (mask != 0).view(n, 1, 1, T)
    s = s.masked_fill(~keep, torch.finfo(torch.float32).min)
    p = torch.softmax(s, dim=-1)
    if drop is not None:
        p = p * attention_dropout_scale(n, n_heads, T, *drop).to(p.device, p.dtype)
    ctx = p @ v  # [n, h, T, dh]
    return ctx.permute(0, 2, 1, 3).reshape(n * T, D)


def backbone_forward(tokens: torch.Tensor, mask: torch.Tensor, params: dict, n_layers: int,
                     n_heads: int, eps: float) -> torch.Tensor:
    """Whole frozen backbone in eval mode -> last hidden state ``[n*T, D]`` (fp32)."""
    x = embed_ln(tokens, params["word"], params["pos"], params["emb_ln_w"], params["emb_ln_b"], eps)
    for i in range(n_layers):
        L = params["layers"][i]
        qkv = linear(x, L["wqkv"], L["bqkv"])
        ctx = title_attention(qkv, mask, n_heads)
        h = linear(ctx, L["wo"], L["bo"], residual=x)
        x = layer_norm(h, L["ln1_w"], L["ln1_b"], eps)
        f = linear(x, L["w1"], L["b1"], act="gelu")
        h = linear(f, L["w2"], L["b2"], residual=x)
        x = layer_norm(h, L["ln2_w"], L["ln2_b"], eps)
    return x


# ---------------------------------------------------------------------------------------
# additive attention pooling (text head and user encoder)
# ---------------------------------------------------------------------------------------
def additive_pool_fwd(x: torch.Tensor, e: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor,
                      literal: bool = False, keep: torch.Tensor | None = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """``x [n,T,D]``, ``e = tanh(W1 x + b1) [n,T,Q]`` -> ``(pooled [n,D], alpha [n,T])``;
    ``keep [n,T]`` (nonzero = pooled) masks positions (mask_padding)."""
    a = _f(e) @ _f(w2).reshape(-1) + _f(b2).reshape(())
    alpha = eps_softmax(a, dim=1, literal=literal, keep=None if keep is None else keep != 0)
    pooled = torch.einsum("nt,ntd->nd", alpha, _f(x))
    return pooled, alpha


def additive_pool_bwd(x: torch.Tensor, e: torch.Tensor, alpha: torch.Tensor, w2: torch.Tensor,
                      g: torch.Tensor):
    """Backward of :func:`additive_pool_fwd` -> ``(dx_direct [n,T,D], de [n,T,Q], dw2 [Q], db2 [])``.

    ``dx_direct`` is the ``alpha_t g`` term only; the ``W1^T dpre`` term is added by the
    caller (``dpre = de * (1 - e^2)``: ``e`` is a tanh output).
    """
    xf, ef, g = _f(x), _f(e), _f(g)
    dalpha = torch.einsum("ntd,nd->nt", xf, g)
    da = eps_softmax_backward(alpha, dalpha, dim=1)
    dx = alpha.unsqueeze(-1) * g.unsqueeze(1)
    de = da.unsqueeze(-1) * _f(w2).reshape(1, 1, -1)
    dw2 = torch.einsum("nt,ntq->q", da, ef)
    db2 = da.sum()
    return dx, de, dw2, db2


# ---------------------------------------------------------------------------------------
# user-side multi-head attention (attention.py:32-82)
# ---------------------------------------------------------------------------------------
def user_attention_fwd(qkv: torch.Tensor, n_heads: int, head_dim: int,
                       literal: bool = False, keep: torch.Tensor | None = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """``qkv [B,H,3*h*d]`` -> ``(ctx [B,H,h*d], A [B,h,H,H])``; ``keep [B,H]`` (nonzero =
    attend) masks keys (mask_padding, attention.py:76-78)."""
    B, H, _ = qkv.shape
    q, k, v = _f(qkv).view(B, H, 3, n_heads, head_dim).permute(2, 0, 3, 1, 4)
    s = q @ k.transpose(-1, -2) / math.sqrt(head_dim)
    A = eps_softmax(s, dim=-1, literal=literal, keep=None if keep is None else (keep != 0).view(B, 1, 1, H))
    ctx = (A @ v).permute(0, 2, 1, 3).reshape(B, H, n_heads * head_dim)
    return ctx, A


def user_attention_bwd(qkv: torch.Tensor, A: torch.Tensor, dctx: torch.Tensor, n_heads: int,
                       head_dim: int) -> torch.Tensor:
    B, H, _ = qkv.shape
    q, k, v = _f(qkv).view(B, H, 3, n_heads, head_dim).permute(2, 0, 3, 1, 4)
    dc = _f(dctx).view(B, H, n_heads, head_dim).permute(0, 2, 1, 3)
    dA = dc @ v.transpose(-1, -2)
    dv = A.transpose(-1, -2) @ dc
    dS = eps_softmax_backward(A, dA, dim=-1) / math.sqrt(head_dim)
    dq = dS @ k
    dk = dS.transpose(-1, -2) @ q
    d = torch.stack([dq, dk, dv], 0)  # [3,B,h,H,d]
    return d.permute(1, 3, 0, 2, 4).reshape(B, H, 3 * n_heads * head_dim)


# ---------------------------------------------------------------------------------------
# scoring + loss (model.py:121-126)
# ---------------------------------------------------------------------------------------
def score_ce_fwd_bwd(cand: torch.Tensor, user: torch.Tensor, act: str = "sigmoid",
                     label: int = 0):
    """Returns ``(loss, scores [B,C], dcand [B,C,D], duser [B,D])`` for a mean CE over the
    batch with target column ``label`` (always 0 in the reference, ``dataset.py:85``)."""
    c, u = _f(cand), _f(user)
    z = torch.einsum("bcd,bd->bc", c, u)
    s = torch.sigmoid(z) if act == "sigmoid" else z
    B = s.shape[0]
    lse = torch.logsumexp(s, dim=1)
    loss = (lse - s[:, label]).mean()
    ds = torch.softmax(s, dim=1)
    ds[:, label] -= 1.0
    ds = ds / B
    dz = ds * s * (1.0 - s) if act == "sigmoid" else ds
    dcand = dz.unsqueeze(-1) * u.unsqueeze(1)
    duser = torch.einsum("bc,bcd->bd", dz, c)
    return loss, s, dcand, duser


# ---------------------------------------------------------------------------------------
# per-news gradient reduction (+ LDP) : client.py:26-48, 87-89; model.py:105-109
# ---------------------------------------------------------------------------------------
def segment_sum_rows(rows: torch.Tensor, inv: torch.Tensor, num_out: int,
                     clip: float = 0.0, noise_std: float = 0.0,
                     generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """``out[inv[r]] += clip_r(rows[r]) + N(0, noise_std)`` -> ``[num_out, D]`` (fp32)."""
    g = _f(rows)
    if clip > 0:
        nrm = g.norm(dim=1, keepdim=True)
        g = g * torch.clamp(clip / (nrm + 1e-12), max=1.0)
    if noise_std > 0:
        g = g + torch.randn(g.shape, generator=generator, device=g.device) * noise_std
    out = torch.zeros(num_out, g.shape[1], dtype=torch.float32, device=g.device)
    out.index_add_(0, inv.long(), g)
    return out


# ---------------------------------------------------------------------------------------
# Adam (torch defaults: no weight decay, no amsgrad; bias correction)
# ---------------------------------------------------------------------------------------
def adam_step(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int,
              lr: float, b1: float, b2: float, eps: float, grad_scale: float = 1.0) -> None:
    gs = g * grad_scale
    m.mul_(b1).add_(gs, alpha=1 - b1)
    v.mul_(b2).addcmul_(gs, gs, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


def title_plan(mask: torch.Tensor):
    """Oracle of the title_count/title_rows kernels: kv rows (mask 1, or every row of an all-masked title)
    first, title-major in position order, then the query-only rows; ``kv_len < 0`` marks an
    all-masked title; ``qstart`` = each title's first query-only row."""
    m = mask.to(torch.int64) != 0
    n, T = m.shape
    allm = ~m.any(1)
    kv = m | allm[:, None]
    cnt = kv.sum(1)
    kv_start = torch.cumsum(cnt, 0) - cnt
    R = int(cnt.sum())
    rank_kv = torch.cumsum(kv.long(), 1) - kv.long()
    rank_q = torch.cumsum((~kv).long(), 1) - (~kv).long()
    q_start = R + torch.arange(n) * T - kv_start
    rowmap = torch.where(kv, kv_start[:, None] + rank_kv, q_start[:, None] + rank_q)
    src = torch.empty(n * T, dtype=torch.int64)
    src[rowmap.reshape(-1)] = torch.arange(n * T)
    kv_len = torch.where(allm, -T * torch.ones_like(cnt), cnt)
    qstart = q_start
    i32 = torch.int32
    return (rowmap.to(i32), src.to(i32), kv_start.to(i32), kv_len.to(i32), qstart.to(i32),
            torch.tensor([R], dtype=i32))
