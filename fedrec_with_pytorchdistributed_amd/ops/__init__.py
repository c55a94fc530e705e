"""Fused ops of the engine.

Device tensors run the hand-written HIP/CDNA4 kernels of ``csrc/`` (``torch.ops.fedrec``);
host tensors run the torch-eager oracle in :mod:`.reference` (the CPU/gloo plumbing
configuration and the numerics reference of the tests).  On a device tensor a missing
extension is an error -- there is no silent eager fallback.

Kernel map:

====================  ===========================  ===========================================
op                    reference site               kernel (csrc/)
====================  ===========================  ===========================================
embed_ln              HF embeddings (K01)          embed_ln.hip: gather + pos add + LayerNorm
linear                q/k/v/out/lin1/lin2, heads   gemm_bf16.hip: MFMA 16x16x32 bf16, fused
                      (K02, K05, K06, K07)         bias / GELU / tanh / residual epilogues
layer_norm            sa/output LN (K04)           layernorm.hip: one wave per row
title_attention       HF attention (K03)           title_attn.hip: MFMA QK^T / PV, T pad 64
title_plan + *_packed frozen-backbone forward      title_attn.hip: pad tokens get Q only (no K/V)
additive_pool_*       attention.py:14-26 (K06/12)  additive_pool.hip: score, eps-softmax, pool
user_attention_*      attention.py:32-82 (K11)     user_attn.hip: 20 heads x d_k 20
score_ce              model.py:121-126 (K13)       score_ce.hip: sigmoid-CE fwd+bwd fused
segment_sum_rows      client.py:26-48,87-89        news_grad.hip: deterministic segment sum
                      (K16, K17)                   + LDP clip + Philox Gaussian noise
adam_flat             model.py:89,93 (K20)         adam.hip: one pass over the flat buffer
dedup / sample_batch  dataset.py:69-86 (K18)       batch.hip: on-device sampling + unique
====================  ===========================  ===========================================
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import native
from . import reference as ref

_ACT = {"none": 0, "gelu": 1, "tanh": 2}


def _dev(t: torch.Tensor) -> bool:
    return t.is_cuda


# ---------------------------------------------------------------------------------------
def embed_ln(tokens, word, pos, ln_w, ln_b, eps: float, dtype=torch.float32):
    if _dev(word):
        if word.dtype != torch.bfloat16:
            native.no_kernel("embed_ln", word)
        return native.require_for(word).embed_ln(tokens.contiguous(), word, pos, ln_w, ln_b, float(eps))
    return ref.embed_ln(tokens, word, pos, ln_w, ln_b, eps).to(dtype)


def linear(x, w, b=None, act: str = "none", residual=None, out_dtype=None):
    """``act(x @ w^T + b) + residual``; bf16 device inputs run the MFMA GEMM."""
    if _dev(x):
        if x.dtype != torch.bfloat16:
            native.no_kernel("linear", x)
        return native.require_for(x).linear(x.contiguous(), w, b, _ACT[act], residual)
    y = ref.linear(x, w, b, act, residual)
    return y.to(out_dtype or x.dtype)


def layer_norm(x, w, b, eps: float, dtype=None, residual=None):
    """``LN(x [+ residual]) * w + b`` (the residual add is fused into the LN kernel)."""
    if _dev(x):
        if x.dtype != torch.bfloat16:
            native.no_kernel("layer_norm", x)
        return native.require_for(x).layer_norm(x, w, b, float(eps), residual)
    h = x if residual is None else x.float() + residual.float()
    return ref.layer_norm(h, w, b, eps).to(dtype or x.dtype)


def title_attention(qkv, mask, n_heads: int, drop=None):
    """``drop = (p, seed, offset)``: train-mode dropout on the attention probabilities."""
    if _dev(qkv):
        if qkv.dtype != torch.bfloat16:
            native.no_kernel("title_attention", qkv)
        if drop is not None:
            p, seed, off = drop
            return native.require_for(qkv).title_attention_drop(qkv, mask.contiguous(), int(n_heads), float(p),
                                                                int(seed), int(off))
        return native.require_for(qkv).title_attention(qkv, mask.contiguous(), int(n_heads))
    return ref.title_attention(qkv, mask, n_heads, drop).to(qkv.dtype)


def title_attention_bwd(qkv, dout, mask, n_heads: int, drop=None):
    lib = native.require_for(qkv)
    if drop is not None:
        p, seed, off = drop
        return lib.title_attention_bwd_drop(qkv, dout.contiguous(), mask.contiguous(), int(n_heads), float(p),
                                            int(seed), int(off))
    return lib.title_attention_bwd(qkv, dout.contiguous(), mask.contiguous(), int(n_heads))


def dropout_add(h, res, p: float, seed: int, offset: int):
    """``res + h o Z`` (``res`` may be None): Z = keep / (1 - p) from the element-indexed
    Philox mask (csrc/dropout.hip).  Its own backward: ``dh = dout o Z``."""
    if _dev(h):
        if h.dtype != torch.bfloat16:
            native.no_kernel("dropout_add", h)
        r = None if res is None else res.contiguous()
        return native.require_for(h).dropout_add(h.contiguous(), r, float(p), int(seed), int(offset))
    return ref.dropout_add(h, res, p, seed, offset).to(h.dtype)


# ---- packed title rows (frozen backbone forward, csrc/title_attn.hip) -----------------------
def title_plan(mask):
    """``mask [n, T]`` -> ``(rowmap [n,T], src [n*T], kv_start [n], kv_len [n], qstart [n], n_kv [1])``:
    the packed row order (key/value rows first, then query-only rows) and its inverse."""
    if _dev(mask):
        return tuple(native.require_for(mask).title_plan(mask.contiguous()))
    return ref.title_plan(mask)


def embed_ln_rows(tokens, src, word, pos, ln_w, ln_b, eps: float):
    """Embedding + LN of packed row r = flat token ``src[r]`` of ``tokens [n, T]``."""
    return native.require_for(word).embed_ln_rows(tokens.contiguous(), src, word, pos, ln_w, ln_b, float(eps))


def linear_split(x, w, b, full_rows, n_partial: int):
    """``x @ w^T + b`` with rows ``>= full_rows[0]`` computed on the first ``n_partial``
    output columns only (the rest of those rows is left unwritten)."""
    return native.require_for(x).linear_split(x.contiguous(), w, b, full_rows, int(n_partial))


def title_attention_packed(qkv, rowmap, kv_start, kv_len, qstart, n_heads: int):
    return native.require_for(qkv).title_attention_packed(qkv, rowmap, kv_start, kv_len, qstart, int(n_heads))


def layer_norm_scatter(x, w, b, eps: float, residual, dst, out=None):
    """``LN(x + residual)`` with row r stored at output row ``dst[r]`` (of ``out`` when given)."""
    return native.require_for(x).layer_norm_scatter(x, w, b, float(eps), residual, dst, out)


def additive_pool_fwd(x, e, w2, b2, keep=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """-> ``(pooled fp32 [n,D], alpha fp32 [n,T])``; ``keep [n,T]`` int (nonzero = pooled):
    the mask_padding position mask."""
    if _dev(x):
        return tuple(native.require_for(x).additive_pool_fwd(x.contiguous(), e.contiguous(),
                                                             w2.reshape(-1).float().contiguous(),
                                                             b2.reshape(-1).float().contiguous(), _mask32(keep)))
    return ref.additive_pool_fwd(x, e, w2, b2, keep=keep)


def _mask32(keep):
    return None if keep is None else keep.to(torch.int32).contiguous()


def additive_pool_bwd(x, e, alpha, w2, g, want_dx: bool, want_colsum: bool = False):
    """-> ``(dx_direct|None, dpre, dw2, db2)`` with ``dpre = da w2 (1 - e^2)`` (tanh folded);
    ``want_colsum`` appends ``dpre`` summed over all tokens (the first linear's bias
    gradient) when the kernel produced it for free, else None."""
    if _dev(x):
        dx, dpre, dw2, db2, dsum = native.require_for(x).additive_pool_bwd(
            x.contiguous(), e.contiguous(), alpha.contiguous(), w2.reshape(-1).float().contiguous(),
            g.float().contiguous(), bool(want_dx))
        out = (dx if want_dx else None), dpre, dw2, db2
        return out + ((dsum if dsum.numel() else None),) if want_colsum else out
    dx, de, dw2, db2 = ref.additive_pool_bwd(x, e, alpha, w2, g)
    dpre = de * (1.0 - e.float() ** 2)
    out = (dx if want_dx else None), dpre, dw2, db2
    return out + (None,) if want_colsum else out


def user_attention_fwd(qkv, heads: int, head_dim: int, keep=None, ctx_b=None):
    """-> ``(ctx [B,H,h*d], saved)``; ``saved`` is whatever the backward needs.  ``keep [B,H]``
    int (nonzero = attend): the mask_padding key mask.  ``ctx_b`` (bf16, like ctx, device
    only): also written with ctx rounded to bf16 (a GEMM operand)."""
    if _dev(qkv):
        return tuple(native.require_for(qkv).user_attention_fwd(qkv.contiguous(), heads, head_dim, _mask32(keep),
                                                                ctx_b))
    out = ref.user_attention_fwd(qkv, heads, head_dim, keep=keep)
    if ctx_b is not None:
        ctx_b.copy_(out[0].reshape(ctx_b.shape))
    return out


def user_qkv_attention_fwd(xd, W, bias, B: int, heads: int, head_dim: int, keep=None, ctx_b=None):
    """Q|K|V projection + attention forward in one launch (device only, H <= 64): ``xd [B*H, Din]``
    bf16, ``W [3*heads*head_dim, Din]`` bf16, ``bias`` fp32 -> ``(ctx [B,H,D], saved, qkv [B,H,3D])``
    -- the values of ``small_gemm(xd, W, +bias)`` followed by :func:`user_attention_fwd`."""
    return tuple(native.require_for(xd).user_qkv_attention_fwd(xd, W, bias, int(B), heads, head_dim, _mask32(keep),
                                                               ctx_b))


def user_attention_bwd_dctx(qkv, saved, dctx, dpre, w1t, heads: int, head_dim: int, keep=None):
    """Attention backward with the additive pool's input-gradient GEMM fused in (device only,
    H <= 64): the attention's dctx is ``dctx + dpre @ w1t.T`` (``dctx`` read, not written; ``dpre
    [B*H, Qd]`` and ``w1t [D, Qd]`` bf16) -> ``dqkv`` bf16 [B, H, 3D]."""
    return native.require_for(qkv).user_attention_bwd_dctx(qkv.contiguous(), saved, dctx.contiguous(), dpre, w1t,
                                                           heads, head_dim, _mask32(keep))


def user_attention_bwd(qkv, saved, dctx, heads: int, head_dim: int, keep=None, bf16_out: bool = False):
    """-> ``dqkv`` like qkv (bf16 with ``bf16_out``: the gradient GEMMs' operand)."""
    if _dev(qkv):
        return native.require_for(qkv).user_attention_bwd(qkv.contiguous(), saved, dctx.contiguous(),
                                                          heads, head_dim, _mask32(keep), bool(bf16_out))
    d = ref.user_attention_bwd(qkv, saved, dctx, heads, head_dim)  # the saved weights hold the mask
    return d.to(torch.bfloat16) if bf16_out else d


def score_ce(cand, user, act: str = "sigmoid"):
    """-> ``(loss [], scores [B,C], dcand [B,C,D], duser [B,D])`` (grads of the mean loss)."""
    if _dev(cand):
        return tuple(native.require_for(cand).score_ce(cand.float().contiguous(), user.float().contiguous(),
                                                       1 if act == "sigmoid" else 0))
    return ref.score_ce_fwd_bwd(cand, user, act)


def score_ce_rows(table, ci, user, act: str, dcand_out):
    """:func:`score_ce` with candidate ``(b, c)`` = row ``ci[b C + c]`` of ``table [U, D]`` and its
    gradient written into ``dcand_out [B C, D]`` -> ``(loss, scores, duser)``."""
    B = user.shape[0]
    if _dev(table):
        loss, scores, _, du = native.require_for(table).score_ce(table, user.contiguous(), 1 if act == "sigmoid" else 0,
                                                                 ci, dcand_out)
        return loss, scores, du
    loss, scores, dcand, du = ref.score_ce_fwd_bwd(table.index_select(0, ci.long()).view(B, -1, table.shape[1]), user,
                                                   act)
    dcand_out.copy_(dcand.reshape(dcand_out.shape))
    return loss, scores, du


def segment_sum_rows(rows, inv, num_out: int, clip: float = 0.0, noise_std: float = 0.0,
                     seed: int = 0, offset: int = 0, generator=None, seg=None, zero_empty: bool = False,
                     dev_off=None):
    """Per-news gradient reduction ``out[inv[r]] += clip(rows[r]) + N(0, noise_std)``.

    ``seg = (perm, seg_ptr)`` (rows grouped by output id) enables the deterministic,
    atomic-free device kernel; it is produced by :func:`dedup`.  The device kernel expects
    the layout dedup produces: every output row has occurrences, except trailing padded rows
    (``zero_empty``, the step graphs' padded unique lists).  ``dev_off`` (device int64[1]):
    added to ``offset`` on the device, so a captured step graph draws fresh noise per replay.
    """
    if _dev(rows):
        if seg is None:
            perm, ptr = segments_from_inv(inv, num_out)
        else:
            perm, ptr = seg
        inv32 = inv.reshape(-1)
        inv32 = inv32 if inv32.dtype == torch.int32 else inv32.to(torch.int32)
        return native.require_for(rows).segment_sum_rows(rows.float().contiguous(), perm, ptr, int(num_out),
                                                         float(clip), float(noise_std), int(seed), int(offset),
                                                         inv32.contiguous(), bool(zero_empty), dev_off)
    if dev_off is not None:
        offset = int(offset) + int(dev_off.reshape(-1)[0])
    if noise_std > 0 and generator is None:
        generator = torch.Generator().manual_seed((int(seed) * 1_000_003 + int(offset)) & 0x7FFFFFFFFFFF)
    return ref.segment_sum_rows(rows, inv, num_out, clip, noise_std, generator)


def segments_from_inv(inv: torch.Tensor, num_out: int):
    inv = inv.reshape(-1).long()
    perm = torch.sort(inv, stable=True).indices.to(torch.int32)
    cnt = torch.bincount(inv, minlength=num_out)
    ptr = torch.zeros(num_out + 1, dtype=torch.int32, device=inv.device)
    ptr[1:] = torch.cumsum(cnt, 0).to(torch.int32)
    return perm, ptr


def adam_flat(p, g, m, v, step: int, lr: float, b1: float, b2: float, eps: float,
              grad_scale: float = 1.0, p_lowp: Optional[torch.Tensor] = None) -> None:
    """One fused Adam step over flat fp32 buffers (torch.optim.Adam semantics)."""
    if _dev(p):
        bc1 = 1.0 - b1 ** step
        bc2 = 1.0 - b2 ** step
        native.require_for(p).adam_flat(p, g, m, v, p_lowp, float(lr), float(b1), float(b2), float(eps),
                                        float(bc1), float(bc2), float(grad_scale))
        return
    ref.adam_step(p, g, m, v, step, lr, b1, b2, eps, grad_scale)
    if p_lowp is not None:
        p_lowp.copy_(p)


def dedup(ids: torch.Tensor, num_news: int):
    """Unique news ids of a batch -> ``(uniq [U], inv [R], perm [R], seg_ptr [U+1])``.

    ``uniq`` is sorted (deterministic), ``inv[r]`` maps each occurrence to its row of
    ``uniq``, ``perm``/``seg_ptr`` group occurrences by row for :func:`segment_sum_rows`.
    """
    flat = ids.reshape(-1)
    if _dev(flat):
        return tuple(native.require_for(flat).dedup(flat.to(torch.int32).contiguous(), int(num_news)))
    uniq, inv = torch.unique(flat.long(), sorted=True, return_inverse=True)
    perm, ptr = segments_from_inv(inv, uniq.numel())
    return uniq.to(torch.int32), inv.to(torch.int32), perm, ptr


# ---- small fp32 GEMMs on MFMA (csrc/small_gemm.hip) ------------------------------------------
class Gemm:
    """One GEMM of a :func:`small_gemm` launch: ``C = act(alpha * A(m,k) B(n,k) + bias) (+C)``.

    ``a_mode`` 0: A row-major [M, K] (``gather_on=1``: row m is ``A[gidx[m]]``); 1: A stored
    [K, M].  ``b_mode`` 0: B [N, K]; 1: B stored [K, N] (``gather_on=2``: row k is
    ``B[gidx[k]]``).  ``drop_on`` 1/2/3: Philox dropout (p, seed, offset) on A elements
    (m, k), on B elements (k, n), or on the output (m, n), element index ``row * drop_ld +
    col`` in the logical (gathered) matrix -- the mask of ``ops.dropout_add``."""

    __slots__ = ("A", "B", "C", "M", "N", "K", "lda", "ldb", "ldc", "a_mode", "b_mode", "act", "accumulate",
                 "alpha", "bias", "gidx", "gather_on", "pdrop", "drop_on", "drop_ld", "seed", "offset", "bseg", "kseg",
                 "asum")

    def __init__(self, A, B, C, M, N, K, lda, ldb, ldc, a_mode=0, b_mode=0, act=0, accumulate=False, alpha=1.0,
                 bias=None, gidx=None, gather_on=0, pdrop=0.0, drop_on=0, drop_ld=0, seed=0, offset=0,
                 bseg=(), kseg=0, asum=None):
        self.A, self.B, self.C = A, B, C
        self.M, self.N, self.K, self.lda, self.ldb, self.ldc = int(M), int(N), int(K), int(lda), int(ldb), int(ldc)
        self.a_mode, self.b_mode, self.act, self.accumulate = int(a_mode), int(b_mode), int(act), bool(accumulate)
        self.alpha, self.bias, self.gidx, self.gather_on = float(alpha), bias, gidx, int(gather_on)
        self.pdrop, self.drop_on, self.drop_ld = float(pdrop), int(drop_on), int(drop_ld)
        self.seed, self.offset = int(seed), int(offset)
        # K-segmented B (b_mode 1): rows [0, kseg) of B, [kseg, 2 kseg) of bseg[0], then bseg[1]
        self.bseg, self.kseg = tuple(bseg), int(kseg)
        # a_mode 1 only: asum[m] = sum_k A(m, k) in fp32 from the raw A values the GEMM stages
        # (a weight gradient's bias gradient dY^T 1 in the same launch)
        self.asum = asum


def gather_dropout(v: torch.Tensor, idx: torch.Tensor, p: float, seed: int, offset: int, dev_off=None,
                   bf16_out: bool = False) -> torch.Tensor:
    """``v[idx] * Z``: rows of ``v`` gathered and dropped out with the counter mask of element
    ``m * K + k`` (offset + ``*dev_off``) -- the mask ``small_gemm``'s dropout loads use.  fp32,
    or bf16 (``bf16_out``: the fp32 product rounded once, as a bf16-operand GEMM would)."""
    if _dev(v):
        return native.require_for(v).gather_dropout(v.contiguous(), idx.to(torch.int32).contiguous(), float(p),
                                                    int(seed), int(offset), dev_off, bool(bf16_out))
    x = v.index_select(0, idx.long())
    if p > 0:
        off = int(offset) + (int(dev_off.item()) if dev_off is not None else 0)
        idx_e = torch.arange(x.numel(), device=x.device, dtype=torch.int64)
        x = x * ref.dropout_scale(idx_e, p, int(seed), off).view_as(x).to(x.dtype)
    return x.to(torch.bfloat16) if bf16_out else x


def small_gemm(*gs: Gemm, dev_off=None, tile: int = 0) -> None:
    """Run up to 6 independent GEMMs in one launch (device only).  ``dev_off``: an int64[1]
    device counter added to every dropout offset (HIP-graph replays draw fresh masks).
    Operands A / B may be fp32 or bf16 (C fp32).  ``tile``: 0 = the launcher's choice, 1..4 =
    64x64 / 128x64 / 64x128 / 128x128, 5 = 64x64 without the LDS-DMA ring of the bf16 x bf16
    k-contiguous launches (benchmarks / tests)."""
    ints, floats, seeds = [], [], []
    for g in gs:
        ints += [g.M, g.N, g.K, g.lda, g.ldb, g.ldc, g.a_mode, g.b_mode, g.act, int(g.accumulate), g.drop_ld,
                 g.drop_on, g.gather_on, g.kseg]
        floats += [g.alpha, g.pdrop]
        seeds += [g.seed, g.offset]
    native.require_for(gs[0].A).small_gemm([g.A for g in gs], [g.gidx for g in gs], [g.B for g in gs],
                                           [g.bias for g in gs], [g.C for g in gs], ints, floats, seeds, dev_off,
                                           [t for g in gs for t in g.bseg], int(tile), [g.asum for g in gs])


def small_gemm_ref(g: Gemm) -> torch.Tensor:
    """fp32 torch emulation of one :class:`Gemm` (operands rounded to bf16 like the kernel)
    -> the new ``C`` [M, N] (tests)."""
    def rows(t, n_rows, n_cols, ld, gidx=None):  # strided view semantics of the kernel (base + r * ld + c)
        flat = torch.as_strided(t, (t.untyped_storage().nbytes() // t.element_size() - t.storage_offset(),), (1,),
                                t.storage_offset())
        idx = gidx.long()[:n_rows] if gidx is not None else torch.arange(n_rows, device=t.device)
        return flat[(idx[:, None] * ld + torch.arange(n_cols, device=t.device)[None, :]).reshape(-1)].view(
            n_rows, n_cols).float()

    def drop(x):  # logical element (r, c) -> index r * drop_ld + c
        idx = (torch.arange(x.shape[0], device=x.device)[:, None] * g.drop_ld
               + torch.arange(x.shape[1], device=x.device)[None, :]).cpu()
        return x * ref.dropout_scale(idx, g.pdrop, g.seed, g.offset).to(x.device)

    A = rows(g.A, g.M, g.K, g.lda, g.gidx if g.gather_on == 1 else None) if g.a_mode == 0 else rows(g.A, g.K, g.M, g.lda).t()
    if g.drop_on == 1:
        A = drop(A)
    if g.b_mode == 0:
        Bm = rows(g.B, g.N, g.K, g.ldb)  # [N, K]
    elif g.kseg:
        Bm = torch.cat([rows(t, min(g.kseg, g.K - i * g.kseg), g.N, g.ldb)
                        for i, t in enumerate((g.B, *g.bseg)) if i * g.kseg < g.K]).t()
    else:
        Bk = rows(g.B, g.K, g.N, g.ldb, g.gidx if g.gather_on == 2 else None)  # [K, N]
        if g.drop_on == 2:
            Bk = drop(Bk)
        Bm = Bk.t()
    A = A.to(torch.bfloat16).float()
    Bm = Bm.to(torch.bfloat16).float()
    out = g.alpha * (A @ Bm.t())
    if g.bias is not None:
        out = out + g.bias.float()[:g.N]
    if g.act == 1:
        out = torch.tanh(out)
    if g.drop_on == 3:
        out = drop(out)
    if g.accumulate:
        out = out + rows(g.C, g.M, g.N, g.ldc)
    return out


def colsum_f32(pairs, accumulate: bool = False) -> None:
    """``out[:N] (+)= X[:M, :N].sum(0)`` for each ``(X, out, M, N, ld)`` (one deterministic launch)."""
    ints = []
    for X, out, M, N, ld in pairs:
        ints += [int(M), int(N), int(ld), int(accumulate)]
    native.require_for(pairs[0][0]).colsum_f32([p[0] for p in pairs], [p[1] for p in pairs], ints)
