"""Autograd wiring of the fused ops.

Each ``Function`` has a hand-written forward *and* backward kernel pair (device) or the
oracle pair (host); torch autograd only strings them together.  Every GEMM of the training
step runs on our MFMA kernels: forward / dX on the NT kernel (``gemm_bf16.hip``), dW on the TN
kernel (``gemm_wgrad.hip``), the fp32 user side on the small-GEMM kernel (``small_gemm.hip``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import math


import torch

from .. import ops
from .reference import _f


def wgrad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """``dy^T x`` in fp32 for ``dy [M, N]``, ``x [M, K]`` with a long reduction dim M.

    On the device with bf16 operands: our TN MFMA kernel (``csrc/gemm_wgrad.hip``: M-major
    tiles staged as they sit in HBM, fragments by LDS transpose reads, split-K over M with a
    fixed-order partial sum)."""
    if not (dy.is_cuda and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16):
        return _f(dy).t() @ _f(x)
    return ops.native.require_for(dy).wgrad(dy.reshape(-1, dy.shape[-1]).contiguous(),
                                            x.reshape(-1, x.shape[-1]).contiguous())


def dgrad(dy: torch.Tensor, wlow: torch.Tensor, residual: Optional[torch.Tensor] = None,
          wt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``dy @ wlow (+ residual)``: the input gradient of ``y = x wlow^T``.

    On the device our NT MFMA GEMM runs it on ``wlow^T`` (a 1-5 MB per-step transpose of the
    bf16 weight; the GEMM streams ~100 MB of ``dy``), with the residual gradient added in the
    epilogue (beta = 1) -- no library GEMM in the training step.  ``wt``: ``wlow^T`` already materialised (the
    unfrozen backbone's pack keeps transposed copies, refreshed once per optimizer step)."""
    if (dy.is_cuda and dy.dtype == torch.bfloat16 and wlow.shape[1] % 128 == 0
            and wlow.shape[0] % 64 == 0):
        return ops.linear(dy, wt if wt is not None else wlow.t().contiguous(), None, residual=residual)
    if residual is not None:
        return residual.addmm_(dy, wlow)
    return torch.mm(dy, wlow)


def bgrad(dy: torch.Tensor) -> torch.Tensor:
    """Column sum in fp32 without materialising an fp32 copy of ``dy`` (bf16 device tensors:
    the two-pass ``colsum`` kernel of ``train_grad.hip``)."""
    if dy.is_cuda and dy.dtype == torch.bfloat16 and dy.shape[-1] % 8 == 0:
        return ops.native.require_for(dy).colsum(dy.reshape(-1, dy.shape[-1]).contiguous())
    return dy.sum(0, dtype=torch.float64 if dy.dtype == torch.float64 else torch.float32)


class AdditivePoolFn(torch.autograd.Function):
    """``AdditiveAttention`` (``attention.py:8-26``): ``x [n,T,D] -> [n,D]``.

    Forward: ``e = tanh(x W1^T + b1)`` (GEMM with a tanh epilogue), then the fused
    score / eps-softmax / weighted-sum kernel.  Backward: the fused kernel yields
    ``alpha g`` and ``dpre = da w2 (1 - e^2)``; ``dW1 = dpre^T x``, ``dx += dpre W1``.
    Device GEMMs: the bf16 NT / TN kernels (text head of the unfrozen backbone) or the
    small-GEMM kernel (fp32 inputs).  ``keep [n,T]`` (optional, nonzero = pooled): the
    mask_padding position mask (masked positions get weight 0).
    """

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, keep=None):
        n, T, D = x.shape
        x2 = x.reshape(n * T, D)
        if x.dtype == torch.bfloat16:  # text head on the device: MFMA GEMM + tanh epilogue
            e = ops.linear(x2, w1.to(x.dtype), b1.float(), act="tanh")
        elif x.is_cuda:  # fp32 on the device: the small MFMA GEMM with a tanh epilogue
            x2 = x2.float().contiguous()
            Q = w1.shape[0]
            e = torch.empty(n * T, Q, device=x.device, dtype=torch.float32)
            ops.small_gemm(ops.Gemm(x2, w1.contiguous(), e, n * T, Q, D, D, D, Q, bias=b1.contiguous(), act=1))
        else:
            e = ops.linear(x2, w1, b1, act="tanh")
        e = e.reshape(n, T, -1)
        pooled, alpha = ops.additive_pool_fwd(x, e, w2, b2, keep)
        ctx.save_for_backward(x, e, alpha, w1, w2)
        return pooled

    @staticmethod
    def backward(ctx, g):
        x, e, alpha, w1, w2 = ctx.saved_tensors
        want_dx = ctx.needs_input_grad[0]
        dx_dir, dpre, dw2, db2, dsum = ops.additive_pool_bwd(x, e, alpha, w2, g, want_dx, want_colsum=True)
        n, T, D = x.shape
        dpre2 = dpre.reshape(n * T, -1)
        x2 = x.reshape(n * T, D)
        dw1 = db1 = None
        small = x2.is_cuda and x2.dtype == torch.float32  # fp32 device: the small MFMA GEMM
        Q = w1.shape[0]
        if small:
            dpre2 = dpre2.contiguous()
            x2 = x2.contiguous()
        if ctx.needs_input_grad[1]:
            if small:  # with the bias gradient (column sums of dpre) from the same launch
                dw1 = torch.empty(Q, D, device=x.device, dtype=torch.float32)
                db1 = torch.empty(Q, device=x.device, dtype=torch.float32)
                ops.small_gemm(ops.Gemm(dpre2, x2, dw1, Q, D, n * T, Q, D, D, a_mode=1, b_mode=1, asum=db1))
            else:
                dw1 = wgrad(dpre2, x2)  # reduced over all n*T tokens (split-K on the device)
        if ctx.needs_input_grad[2] and db1 is None:
            if dsum is not None:
                db1 = dsum
            elif small:
                db1 = torch.empty(Q, device=x.device, dtype=torch.float32)
                ops.colsum_f32([(dpre2, db1, n * T, Q, Q)])
            else:
                db1 = bgrad(dpre2)
        dx = None
        if want_dx:
            if small:  # dx = alpha g + dpre W1, the GEMM accumulating onto the direct term
                dx = dx_dir.float().contiguous()
                ops.small_gemm(ops.Gemm(dpre2, w1.contiguous(), dx.view(n * T, D), n * T, D, Q, Q, D, D, b_mode=1,
                                        accumulate=True))
            else:
                if x2.is_cuda and x2.dtype == torch.bfloat16:
                    dxp = dgrad(dpre2.contiguous(), w1.to(torch.bfloat16))
                else:
                    dxp = _f(dpre2) @ _f(w1)
                dx = (_f(dx_dir) + dxp.reshape(n, T, D)).to(x.dtype)
        return dx, dw1, db1, dw2.reshape(1, -1).to(w2.dtype), db2.reshape(1).to(w2.dtype), None


# N > 1 (the engine, around a step's forward + backward): the text head's and its fc's weight
# gradients go straight into their slots of the flat gradient buffer -- the gradient all-reduce
# reads them there, and the end-of-backward copy of the six fresh tensors (one launch on the
# critical path between the backward and the head slice's all-reduce) is gone.  ``_GRAD_INTO``
# maps id(parameter) -> its flat slot (a view of the parameter's shape); a Function whose weights
# all have slots writes them in place, returns None for them and records them in
# ``_GRAD_WRITTEN``, which the engine hands to ``FlatParams.end_backward`` (slots not to zero).
_GRAD_INTO: dict = {}
_GRAD_WRITTEN: set = set()


class grads_into:
    """Context: the weight-gradient destinations of :data:`_GRAD_INTO` for the backward run inside it."""

    def __init__(self, mapping: dict):
        self.mapping = mapping

    def __enter__(self):
        _GRAD_INTO.clear()
        _GRAD_INTO.update(self.mapping)
        _GRAD_WRITTEN.clear()
        return self

    def __exit__(self, *exc):
        _GRAD_INTO.clear()
        return False


def take_written() -> set:
    """ids of the parameters whose gradients a backward wrote in place (and forget them)."""
    out = set(_GRAD_WRITTEN)
    _GRAD_WRITTEN.clear()
    return out


def _slots(*params):
    """The flat-gradient slots of ``params`` (all of them, fp32 contiguous), else None."""
    if not _GRAD_INTO:
        return None
    out = []
    for p in params:
        v = _GRAD_INTO.get(id(p))
        if v is None or v.dtype != torch.float32 or not v.is_contiguous() or v.shape != p.shape:
            return None
        out.append(v)
    return tuple(out), tuple(id(p) for p in params)


class TextHeadFn(torch.autograd.Function):
    """The text head's attention pooling (``encoder.py:27-28`` -> ``attention.py:14-26``) over
    GATHERED hidden states: rows of ``table [rows, D]`` (the HBM hidden-state cache, or a
    batch's hidden states) picked by title index ``ids [U]`` (None: titles 0..U-1), ``T`` tokens
    per title -> pooled ``[U, D]`` fp32 (the ``fc`` follows as :class:`HeadFCFn`).

    ``csrc/text_head.hip``: forward = the att_fc1 GEMM with its A rows loaded by index and a
    tanh.w2 row-dot epilogue (scores a; e kept in bf16 for the backward) + the per-title pool;
    backward = the pool backward (da) + the att_fc1 weight gradient with
    ``dpre = da w2 (1 - e^2)`` formed inside its LDS pipeline, with the db1 / dw2 / db2 sums.
    No hidden-state gather, no dpre tensor.  The hidden states get no gradient (frozen
    backbone); the unfrozen backbone keeps :class:`AdditivePoolFn`.  ``tokens [N, 2, T]``
    int32 (optional, indexed like the table's titles): padding tokens get weight 0 (the
    ``mask_padding`` option, Q7)."""

    @staticmethod
    def forward(ctx, w1, b1, w2, b2, table, ids, T: int, tokens, nreal=None, w1b=None, want_bf16=False):
        # nreal (device int32 [1], optional): titles past it are padding of a step graph's unique
        # list -- every kernel skips them (pooled / da exactly 0, no rows in the weight gradient).
        # want_bf16: also returns pooled rounded to bf16 (non-differentiable) -- the fc GEMMs'
        # operand, the rounding they would apply to the fp32 rows themselves
        lib = ops.native.require_for(table)
        need = any(ctx.needs_input_grad[:4])
        w1c = w1b if w1b is not None else w1.to(torch.bfloat16).contiguous()  # w1b: the step's cast
        e, a = lib.head_score(table, ids, T, w1c, b1.contiguous(),
                              w2.reshape(-1).contiguous(), b2.reshape(-1), need, nreal)
        pooled, alpha, pooled_b = lib.head_pool(table, ids, T, a, tokens, nreal, bool(want_bf16))
        if need:
            ctx.save_for_backward(table, ids, e, alpha, w2, nreal)
        ctx.T = T
        ctx.into = _slots(w1, b1, w2, b2) if all(ctx.needs_input_grad[:4]) else None
        ctx.mark_non_differentiable(pooled_b)
        # no zero tensor for pooled_b's (never used) gradient: autograd would otherwise fill one
        # [U, D] bf16 buffer per backward (a 5.5 us fill launch in every config-2 step)
        ctx.set_materialize_grads(False)
        return pooled, pooled_b

    @staticmethod
    def backward(ctx, g, g_b=None):
        table, ids, e, alpha, w2, nreal = ctx.saved_tensors
        lib = ops.native.require_for(table)
        if g is None:
            g = torch.zeros(ids.numel(), table.shape[-1], device=table.device)
        if _head_g_path(table.shape[-1], w2.numel(), ctx.T):
            # the G path: the pool backward also turns e into g = da (1 - e^2) (in place) with the
            # per-title column sums, and the weight gradient is a plain TN GEMM over g
            da, db2p, cs = lib.head_pool_bwd_g(table, ids, ctx.T, alpha, g.contiguous().float(), e, nreal)
            if ctx.into is not None:  # into the flat gradient's slots (N > 1): no fresh tensors to copy
                views, pids = ctx.into
                lib.head_wgrad_g(table, ids, ctx.T, e, cs, w2.reshape(-1).contiguous(), db2p, nreal,
                                 [v.view(-1) for v in views])
                _GRAD_WRITTEN.update(pids)
                return None, None, None, None, None, None, None, None, None, None, None
            dw1, db1, dw2, db2 = lib.head_wgrad_g(table, ids, ctx.T, e, cs, w2.reshape(-1).contiguous(), db2p, nreal)
        else:
            da, db2p = lib.head_pool_bwd(table, ids, ctx.T, alpha, g.contiguous().float(), nreal)
            dw1, db1, dw2, db2 = lib.head_wgrad(table, ids, ctx.T, e, da, w2.reshape(-1).contiguous(), db2p, nreal)
        return dw1, db1, dw2.view(1, -1), db2.view(1), None, None, None, None, None, None, None


_HEAD_G: dict = {}


def _head_g_path(D: int, Q: int, T: int) -> bool:
    """The text head's backward on the G path (``head_pool_bwd_g``: pool backward + the g
    rewrite in one launch, 52.4 us vs 27.8 + 22.7 us as two; then ``head_wgrad_g``) where the
    shape allows (Q = 384, the DistilBERT head); other head widths (Q = 128 / 256: the tiny test
    backbones) keep the round-4 path (the e -> g rewrite inside ``head_wgrad``)."""
    key = (int(D), int(Q), int(T))
    if key not in _HEAD_G:
        _HEAD_G[key] = bool(ops.native.lib().head_g_supported(*key))
    return _HEAD_G[key]


# the fused text head over the cache (head_score2 / head_pool2 / G path) wherever the shape allows;
# False only in tests that compare against the round-2 path (gather + GEMM + AdditivePoolFn)
FUSED_HEAD = True


def fused_head_supported(table_dim: int, query_dim: int, title_len: int) -> bool:
    """Shapes the fused text-head kernels take (D % 256 == 0, Q in {128, 256, 384}, T <= 128)."""
    if not FUSED_HEAD:
        return False
    return bool(ops.native.lib().head_supported(int(table_dim), int(query_dim), int(title_len)))


class UserAttentionFn(torch.autograd.Function):
    """``ScaledDotProductAttention`` over 20 heads x d_k 20 (``attention.py:32-82``); ``keep
    [B,H]`` (optional, nonzero = attend): the mask_padding key mask."""

    @staticmethod
    def forward(ctx, qkv, heads: int, head_dim: int, keep=None):
        out, saved = ops.user_attention_fwd(qkv, heads, head_dim, keep)
        ctx.save_for_backward(qkv, saved)
        ctx.heads, ctx.head_dim, ctx.keep = heads, head_dim, keep
        return out

    @staticmethod
    def backward(ctx, dctx):
        qkv, saved = ctx.saved_tensors
        return ops.user_attention_bwd(qkv, saved, dctx, ctx.heads, ctx.head_dim, ctx.keep), None, None, None


class ScoreCEFn(torch.autograd.Function):
    """``CE(sigmoid(<cand, u>), 0)`` with the gradients computed in the same kernel."""

    @staticmethod
    def forward(ctx, cand, user, act: str = "sigmoid"):
        loss, scores, dcand, duser = ops.score_ce(cand, user, act)
        ctx.save_for_backward(dcand, duser)
        ctx.mark_non_differentiable(scores)
        return loss, scores

    @staticmethod
    def backward(ctx, gloss, gscores):
        dcand, duser = ctx.saved_tensors
        return dcand * gloss, duser * gloss, None


class NewsGatherFn(torch.autograd.Function):
    """Rows of the per-batch news table for every candidate/history occurrence.

    Backward is the per-news gradient reduction of the reference (``client.py:26-48``,
    ``model.py:105-109``) with the optional LDP step (``client.py:87-89``) fused in:
    per-occurrence clip + Gaussian noise, then a deterministic segment sum.
    """

    @staticmethod
    def forward(ctx, table, inv, perm, seg_ptr, clip: float, noise_std: float, seed: int, offset: int,
                padded: bool = False):
        ctx.save_for_backward(inv, perm, seg_ptr)
        ctx.n = table.shape[0]
        ctx.ldp = (clip, noise_std, seed, offset)
        ctx.padded = padded  # table rows no occurrence maps to (step graphs): their gradient is 0
        return table.index_select(0, inv.long())

    @staticmethod
    def backward(ctx, g):
        inv, perm, seg_ptr = ctx.saved_tensors
        clip, noise, seed, offset = ctx.ldp
        d = ops.segment_sum_rows(g, inv, ctx.n, clip, noise, seed, offset, seg=(perm, seg_ptr), zero_empty=ctx.padded)
        return d, None, None, None, None, None, None, None, None


def additive_pool(x, lin1: torch.nn.Linear, lin2: torch.nn.Linear, keep=None):
    return AdditivePoolFn.apply(x, lin1.weight, lin1.bias, lin2.weight, lin2.bias, keep)


def user_attention(qkv, heads: int, head_dim: int, keep=None):
    return UserAttentionFn.apply(qkv, heads, head_dim, keep)


# padding masks (config mask_padding): the reference passes mask=None everywhere,
# but its AdditiveAttention / ScaledDotProductAttention take an optional mask that multiplies
# exp(score) before the +1e-8 normalisation (attention.py:20-22, 40-42).  Every pool /
# attention above takes it as ``keep`` (kernels on the device, ops/reference.py on the host):
# masked positions get weight exactly 0, a fully masked row gives 0.


def score_ce(cand, user, act: str = "sigmoid") -> Tuple[torch.Tensor, torch.Tensor]:
    return ScoreCEFn.apply(cand, user, act)


def news_gather(table, inv, perm, seg_ptr, clip: float = 0.0, noise_std: float = 0.0,
                seed: int = 0, offset: int = 0, padded: bool = False):
    return NewsGatherFn.apply(table, inv, perm, seg_ptr, clip, noise_std, seed, offset, padded)


# ---------------------------------------------------------------------------------------
# training-mode backbone (unfrozen encoder, BASELINE config 5): forward on the fp32 master
# parameters through their bf16 compute copies; backward kernels for attention / LayerNorm /
# GELU, our NT GEMM for dX (``dgrad``) and our TN GEMM for dW (``wgrad``).
# ---------------------------------------------------------------------------------------
class DropoutFn(torch.autograd.Function):
    """Train-mode dropout with the counter-based mask (``ops.dropout_add``): the backward
    regenerates Z from (seed, offset) instead of storing it."""

    @staticmethod
    def forward(ctx, x, p: float, seed: int, offset: int):
        ctx.drop = (p, seed, offset)
        return ops.dropout_add(x, None, p, seed, offset)

    @staticmethod
    def backward(ctx, g):
        return ops.dropout_add(g.contiguous(), None, *ctx.drop), None, None, None


class AttnBlockFn(torch.autograd.Function):
    """``h = out_proj(attention(x Wqkv^T + bqkv)) + x`` (one post-LN block's attention half,
    unfrozen backbone).  One Function so the residual gradient joins the QKV input gradient
    inside the dgrad GEMM (``dqkv Wqkv + dh`` in the GEMM epilogue: beta = 1) instead of an
    extra bf16 add pass over [M, 768] that autograd would insert for the two uses of ``x``.
    ``drop = (p, seed, offset)``: train-mode dropout of the attention probabilities (HF
    DistilBERT has no dropout after ``out_lin``)."""

    @staticmethod
    def forward(ctx, x, wq, wk, wv, bq, bk, bv, wo, bo, mask, heads: int, wqkv_low, bqkv, wo_low, box=None,
                drop=None, wts=(None, None)):
        # wq .. bv: the fp32 masters (autograd inputs: their gradients are slices of dwqkv /
        # dbqkv, so no per-step fp32 cat of the three weights); the GEMM runs on the fused bf16
        # compute copy wqkv_low and the fused fp32 bias bqkv of the backbone's pack
        qkv = ops.linear(x, wqkv_low, bqkv)
        c = ops.title_attention(qkv, mask, heads, drop)
        h = ops.linear(c, wo_low, bo, residual=x)
        ctx.save_for_backward(x, qkv, c, mask, wqkv_low, wo_low, wo)
        ctx.heads = heads
        ctx.box = box
        ctx.drop = drop
        ctx.wts = wts  # (Wqkv^T, Wo^T) bf16 or None: not saved tensors (refreshed in place per step)
        return h

    @staticmethod
    def backward(ctx, dh):
        x, qkv, c, mask, wqkv_low, wo_low, wo = ctx.saved_tensors
        wqkv_t, wo_t = ctx.wts
        dh = dh.contiguous()
        dbo = ctx.box.pop("colsum", None) if ctx.box is not None else None  # from LN1's backward
        dwo, dbo = wgrad(dh, c), (dbo if dbo is not None else bgrad(dh))
        dc = dgrad(dh, wo_low, wt=wo_t)
        dqkv = ops.title_attention_bwd(qkv, dc, mask, ctx.heads, ctx.drop)
        dwqkv = wgrad(dqkv, x)
        if dqkv.is_cuda and ctx.drop is None:
            # column sums of dQ | dK | dV without reading dK and dV: every softmax row sums to
            # one, so sum_s dV_s = sum_t dctx_t = dbo Wo; and sum_s dS_ts = 0 for every query
            # (shift invariance), so the key-bias gradient is identically zero.  (Not with
            # attention dropout: the dropped rows of P~ no longer sum to one.)
            Dm = wo.shape[0]
            dbqkv = torch.cat([ops.native.require_for(dqkv).colsum(dqkv[:, :Dm]),
                               torch.zeros(Dm, device=dqkv.device, dtype=torch.float32),
                               (dbo.float().unsqueeze(0) @ wo.float()).squeeze(0)])
        elif dqkv.is_cuda:
            # with attention dropout the key-bias gradient is still exactly zero (the dropout
            # acts after the softmax: sum_s dS_ts = D_t - D_t sum_s P_ts = 0), but the dropped
            # P~ rows no longer sum to one, so dV needs its own column sums
            Dm = wo.shape[0]
            lib = ops.native.require_for(dqkv)
            dbqkv = torch.cat([lib.colsum(dqkv[:, :Dm]), torch.zeros(Dm, device=dqkv.device, dtype=torch.float32),
                               lib.colsum(dqkv[:, 2 * Dm:])])
        else:
            dbqkv = bgrad(dqkv)
        dx = dgrad(dqkv, wqkv_low, residual=dh, wt=wqkv_t)  # residual + QKV dgrad in one GEMM (beta = 1)
        Dm = dwqkv.shape[0] // 3
        dw = [dwqkv[i * Dm:(i + 1) * Dm] for i in range(3)]
        db = [dbqkv[i * Dm:(i + 1) * Dm] for i in range(3)]
        return (dx, *dw, *db, dwo, dbo) + (None,) * 8


class MLPBlockFn(torch.autograd.Function):
    """``h = drop(GELU(x W1^T + b1) W2^T + b2) + x`` (FFN half of a block, unfrozen backbone;
    ``drop = (p, seed, offset)`` = HF ``FFN.dropout`` in train mode, else identity).
    Backward: the GELU derivative rides in the epilogue of the GEMM that forms dF
    (``act = 3``: ``dz = (dh W2) * GELU'(z)``, z saved by the dual-store forward GEMM), and
    the residual gradient joins the FFN1 dgrad in its GEMM epilogue (beta = 1)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w1_low, w2_low, box=None, drop=None, wts=(None, None)):
        lib = ops.native.require_for(x)
        if box is not None and drop is not None:
            box["drop"] = drop  # LN2's backward applies this dropout's backward in its own pass
        f, z = lib.linear_gelu_dual(x.contiguous(), w1_low, b1)
        if drop is None:
            h = ops.linear(f, w2_low, b2, residual=x)
        else:  # dropout + residual in one elementwise pass over the lin2 output
            h = ops.dropout_add(ops.linear(f, w2_low, b2), x, *drop)
        ctx.save_for_backward(x, f, z, w1_low, w2_low)
        ctx.box = box
        ctx.drop = drop
        ctx.wts = wts  # (W1^T, W2^T) bf16 or None
        return h

    @staticmethod
    def backward(ctx, dh):
        x, f, z, w1_low, w2_low = ctx.saved_tensors
        lib = ops.native.require_for(x)
        dres = dh.contiguous()  # the residual branch's gradient
        db2 = ctx.box.pop("colsum", None) if ctx.box is not None else None  # from LN2's backward
        dz2 = ctx.box.pop("dxz", None) if ctx.box is not None else None
        if ctx.drop is not None and dz2 is not None:
            dh = dz2  # dh o Z and its column sums (db2) came out of LN2's backward pass
        elif ctx.drop is not None:  # the lin2 branch sees dh o Z; LN2's column sums are of dh itself
            dh, db2 = ops.dropout_add(dres, None, *ctx.drop), None
        else:
            dh = dres
        dw2, db2 = wgrad(dh, f), (db2 if db2 is not None else bgrad(dh))
        # (dh W2) * GELU'(z) and its column sums from our GEMM's epilogue in one pass (the
        # aux-input epilogue makes that GEMM 650 us vs 480 for the forward FFN1 shape; a separate
        # streaming pass measured the same step time: bench_r1_cfg5_dzmode_ab.jsonl)
        w2t = ctx.wts[1] if ctx.wts[1] is not None else w2_low.t().contiguous()
        dz, db1 = lib.linear_gelu_bwd(dh, w2t, z)
        if db1 is None:
            db1 = bgrad(dz)
        dw1 = wgrad(dz, x)
        dx = dgrad(dz, w1_low, residual=dres, wt=ctx.wts[0])
        return dx, dw1, db1, dw2, db2, None, None, None, None, None


class LayerNormFn(torch.autograd.Function):
    """``box`` (optional dict): the backward also leaves the column sums of its dx in
    ``box["colsum"]`` -- the bias gradient of the block Function that produced the LN input
    and runs its backward right after (one pass instead of a separate colsum over dx)."""

    @staticmethod
    def forward(ctx, x, w, b, eps: float, box=None):
        ctx.save_for_backward(x, w)
        ctx.eps = eps
        ctx.box = box
        return ops.layer_norm(x, w, b, eps)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        lib = ops.native.require_for(x)
        drop = ctx.box.pop("drop", None) if ctx.box is not None else None
        if drop is not None:
            p, seed, off = drop
            dx, ctx.box["dxz"], dw, db, ctx.box["colsum"] = lib.layer_norm_bwd_drop(
                x.contiguous(), w, dy.contiguous(), float(ctx.eps), float(p), int(seed), int(off))
        elif ctx.box is not None:
            dx, dw, db, ctx.box["colsum"] = lib.layer_norm_bwd_colsum(x, w, dy.contiguous(), float(ctx.eps))
        else:
            dx, dw, db = lib.layer_norm_bwd(x, w, dy.contiguous(), float(ctx.eps))
        return dx, dw, db, None, None


class EmbedLNFn(torch.autograd.Function):
    """``LN(word[tok] + pos[t])``; backward = LN backward, then a scatter-add into the word
    table rows and a per-position sum into the position table."""

    @staticmethod
    def forward(ctx, tokens, word, pos, w, b, eps: float, word_low, pos_low):
        ctx.save_for_backward(tokens, word_low, pos_low, w)
        ctx.eps = eps
        ctx.shapes = (word.shape, pos.shape)
        return ops.embed_ln(tokens, word_low, pos_low, w, b, eps)

    @staticmethod
    def backward(ctx, dy):
        tokens, word_low, pos_low, w = ctx.saved_tensors
        n, T = tokens.shape
        x0 = (word_low.index_select(0, tokens.reshape(-1).long()).view(n, T, -1) + pos_low[:T].unsqueeze(0))
        x0 = x0.reshape(n * T, -1).contiguous()
        dx0, dw, db = ops.native.require_for(x0).layer_norm_bwd(x0, w, dy.contiguous(), float(ctx.eps))
        flat_tok = tokens.reshape(-1)
        if dx0.is_cuda and dx0.dtype == torch.bfloat16 and dx0.shape[1] % 256 == 0:
            # sort-based, deterministic, skips the pad token (most rows): no atomic hot spot
            srt, perm = torch.sort(flat_tok.to(torch.int32), stable=True)
            dword = ops.native.require_for(dx0).embed_grad(dx0, srt.to(torch.int32), perm.to(torch.int32),
                                                            ctx.shapes[0][0])
        else:
            dword = torch.zeros(ctx.shapes[0], dtype=torch.float32, device=dy.device)
            dword.index_add_(0, flat_tok.long(), dx0.float())
        dword[0] = 0.0  # nn.Embedding(padding_idx=0): the pad row never receives gradient
        dpos = torch.zeros(ctx.shapes[1], dtype=torch.float32, device=dy.device)
        dpos[:T] = bgrad(dx0.view(n, -1)).view(T, -1)  # per-position sum over titles
        return None, dword, dpos, dw, db, None, None, None


# ---------------------------------------------------------------------------------------
# the device user side of a step as ONE autograd Function:
# candidate gather -> [gather + dropout + Q|K|V projection] -> user attention -> additive
# pool -> sigmoid-CE, and a hand-written backward.  Every GEMM is csrc/small_gemm.hip, every
# bias gradient the deterministic colsum, the per-news reduction (+ LDP) the segment sum.
# ---------------------------------------------------------------------------------------


def _user_weight_bufs(wts, dev, transposed: bool = False):
    """The user step's compute copies: the bf16 stack [Wq; Wk; Wv; W1], the fp32 [bq | bk | bv]
    and (``transposed``) W1^T ``[D, Qd]`` bf16: the dctx GEMM's weight k-contiguous (the
    register-direct small GEMM).  (The Q|K|V input gradient stays on the LDS-DMA ring over the
    stored weight: register-direct on a cast W^T measured slower there.)"""
    wq, w1, D = wts[0], wts[6], wts[0].shape[1]
    bufs = (torch.empty(3 * wq.shape[0] + w1.shape[0], D, device=dev, dtype=torch.bfloat16),
            torch.empty(3 * wq.shape[0], device=dev, dtype=torch.float32))
    if transposed:
        bufs += (torch.empty(D, w1.shape[0], device=dev, dtype=torch.bfloat16),)
    return bufs


def _user_cast_lists(wts, wb, bqkv, wbt=None):
    wq, bq, wk, bk, wv, bv, w1 = wts[:7]
    D, D3 = wq.shape[1], 3 * wq.shape[0]
    src = [wq, wk, wv, w1, bq, bk, bv]
    dst = [wb[:D], wb[D:2 * D], wb[2 * D:D3], wb[D3:], bqkv[:D], bqkv[D:2 * D], bqkv[2 * D:]]
    if wbt is not None:  # a transposed view: the cast launch writes W1^T (multi_cast T segment)
        src.append(w1)
        dst.append(wbt.t())
    return src, dst


def _step_cast_weights(text_encoder, user_encoder):
    aa = text_encoder.additive_attention
    mha, pool = user_encoder.multihead_attention, user_encoder.additive_attention
    wts = (mha.W_Q.weight, mha.W_Q.bias, mha.W_K.weight, mha.W_K.bias, mha.W_V.weight, mha.W_V.bias,
           pool.att_fc1.weight)
    return aa.att_fc1.weight, text_encoder.fc.weight, wts


def step_cast_buffers(text_encoder, user_encoder):
    """The compute copies :func:`step_weight_casts` fills: ``(w1_bf16, (wb, bqkv, wbt), (fc_bf16,
    fc_bf16^T))`` -- the transposed copies are the input-gradient GEMMs' k-contiguous weights."""
    w, wf, wts = _step_cast_weights(text_encoder, user_encoder)
    w1b = torch.empty(w.shape, device=w.device, dtype=torch.bfloat16)
    fcb = torch.empty(wf.shape, device=w.device, dtype=torch.bfloat16)
    return w1b, _user_weight_bufs(wts, w.device, transposed=True), (fcb, None)


def step_cast_lists(text_encoder, user_encoder, bufs):
    """``(sources, destinations)`` of the step's weight casts into ``bufs`` (step_cast_buffers)."""
    w, wf, wts = _step_cast_weights(text_encoder, user_encoder)
    w1b, (wb, bqkv, wbt), (fcb, fcbt) = bufs
    src, dst = _user_cast_lists(wts, wb, bqkv, wbt)
    src, dst = [w.detach(), wf.detach()] + [t.detach() for t in src], [w1b, fcb] + dst
    return src, dst


def step_weight_casts(text_encoder, user_encoder, bump=None, bump2=None):
    """Every compute copy a fused training step needs, in ONE cast launch: the text head's att_fc1
    weight in bf16 (the head_score operand), its fc weight in bf16 (the fc GEMMs' operand) and the
    user encoder's bf16 weight stack + fp32 Q|K|V bias (the user step's GEMM operands), with the
    transposed copies of the user and fc weights.  Returns ``(w1_bf16, (wb, bqkv, wbt), (fc_bf16,
    fc_bf16^T))``; the att_fc1 and user casts were a cast
    kernel each (4.7 + 6.2 us per step).  ``bump`` (int64 [1] device counter, optional): advanced
    by one in the same launch -- the step's dropout / noise offset (a torch ``add_`` of its own
    cost 4.8 us at the end of every step).  ``bump2``: a second counter advanced the same way (the
    in-graph Adam's step count: adam_dev then only reads it).  A captured step graph takes these
    copies from persistent buffers its replay's input launch fills instead (engine _StepGraph)."""
    bufs = step_cast_buffers(text_encoder, user_encoder)
    src, dst = step_cast_lists(text_encoder, user_encoder, bufs)
    launched = ops.native.require_for(dst[0]).multi_cast(src, dst, bump, bump2)
    if not launched:
        for b in (bump, bump2):
            if b is not None:
                b.add_(1)
    return bufs


# register-direct small-GEMM variants (csrc/small_gemm.hip tile codes 1000 + 10 f + P) per
# call site, measured on the config-2 shapes in the step graph (profiles/r5n_sg_rd.jsonl); a
# launch whose operands the form does not take falls back to the automatic choice
RD_ATT_FC1 = 1002  # 32 x 32 waves, 2 k-steps in flight
RD_DCTX = 1004

# the user encoder's Q|K|V projection fused into the attention forward launch and the additive
# pool's input-gradient GEMM into the attention backward launch (user_attn.hip) where the shape
# allows (H <= 64, d_k = 20); False only in tests comparing against the separate launches
FUSED_QKV_ATTN = True

# (Measured and not kept, round 5: the weight-gradient GEMMs forked onto a side stream beside
# the rest of the backward -- steady 0.539-0.549 vs 0.491-0.494 ms; every kernel the side work
# overlapped slowed down, docs/PERFORMANCE.md.  The user encoder's weight gradients are instead
# held back to ride in the text fc's backward launch.)
_SIDE_DEPTH = [0]
_PENDING_GEMMS: list = []


def _flush_pending_gemms() -> None:
    if _PENDING_GEMMS:
        gs = list(_PENDING_GEMMS)
        _PENDING_GEMMS.clear()
        ops.small_gemm(*gs)


def take_pending_gemms(room: int) -> list:
    """Up to ``room`` pending weight-gradient GEMMs for a launch of the caller's (all of them or
    none: they share a launch)."""
    if not _PENDING_GEMMS or len(_PENDING_GEMMS) > room:
        return []
    gs = list(_PENDING_GEMMS)
    _PENDING_GEMMS.clear()
    return gs


# Deferred split-K reduction (inside side_wgrads, i.e. the engine's step without a bucket reducer:
# no gradient hook reads a weight gradient before the backward ends).  The text fc's backward
# launch (its input gradient + the fc and user-encoder weight gradients) leaves the split-K
# reduction of its weight gradients pending, and the text head's reduce launch runs it in extra
# blocks (csrc/text_head.hip head_reduce_kernel<true>): one launch fewer per step.  Whatever is
# still pending when the context ends is reduced then.  False only in the tests comparing
# against the standalone reduce.
DEFER_REDUCE = True
_DEFERRED = [False]

# Early gradient reduction at N > 1 (DDP's bucket that fires inside the backward): while a step
# graph with an in-graph all-reduce is captured, the engine sets this callback; the text fc's
# backward launch -- the one that also computes the held-back user-encoder weight gradients --
# calls it right after that launch (its split-K reduce then runs at once, not deferred), so the
# user-encoder slice of the flat gradient is summed over the clients on a side stream while the
# text-head backward still runs (train/engine.py LocalEngine._early_user_reduce).
_AFTER_USER_WGRADS = [None]


class after_user_wgrads:
    """Context: ``cb()`` runs once the user encoder's weight gradients are final in a backward."""

    def __init__(self, cb):
        self.cb = cb

    def __enter__(self):
        _AFTER_USER_WGRADS[0] = self.cb
        return self

    def __exit__(self, *exc):
        _AFTER_USER_WGRADS[0] = None
        return False


def defer_active() -> bool:
    return DEFER_REDUCE and _SIDE_DEPTH[0] > 0


class side_wgrads:
    """Context: the engine's training step (no bucket reducer): backwards run inside it leave
    their weight gradients' split-K reduction to a later launch (DEFER_REDUCE); on exit nothing
    is left pending."""

    def __enter__(self):
        _SIDE_DEPTH[0] += 1
        return self

    def __exit__(self, *exc):
        _SIDE_DEPTH[0] -= 1
        if _SIDE_DEPTH[0] == 0 and _DEFERRED[0]:
            _DEFERRED[0] = False
            ops.native.lib().small_gemm_flush_pending()
        return False


def _user_enc_fwd(src, idx, wts, B: int, H: int, heads: int, hd: int, drop, dev_off, keep, casts=None,
                  pool: bool = True):
    """Device user encoder forward over history rows ``src[idx]`` (``src [*, D]`` fp32, ``idx``
    int32 [B*H]) -> ``(u [B, D] fp32, saved)``.

    The input dropout (``encoder.py:50``) is the Philox mask of element ``(b*H + t) * D + d`` of
    the gathered history matrix with offset ``drop[2] + *dev_off``: X' = drop(src[idx]) is
    materialised once in bf16 (``ops.gather_dropout``, 2.5 MB at config 2) and read by the
    Q|K|V GEMM and the weight gradients; the dgrad regenerates the mask in its epilogue.  The
    GEMM weights go through one bf16 stack [Wq; Wk; Wv; W1] (one cast launch; what the GEMMs'
    fp32 loads rounded to).  ``keep [B, H]`` int32 (nonzero = real history slot, or None): the
    mask_padding key mask of the attention and the pool (attention.py:76-78)."""
    wq, bq, wk, bk, wv, bv, w1, b1, w2, b2 = wts
    D = src.shape[1]
    BH, D3, Qd = B * H, 3 * D, w1.shape[0]
    dev = src.device
    wbt = None
    if casts is not None:  # the step's one cast launch made them already (step_weight_casts)
        wb, bqkv, *rest = casts
        wbt = rest[0] if rest else None
    else:
        wb, bqkv = _user_weight_bufs(wts, dev)
        ops.native.require_for(src).multi_cast(*_user_cast_lists(wts, wb, bqkv))
    p, seed, off = drop
    xd = ops.gather_dropout(src, idx, p, seed, off, dev_off, bf16_out=True)
    # the attention also writes ctx rounded to bf16 -- what the att_fc1 GEMM and dW1 would round
    # it to on their loads -- so both run as bf16 x bf16 launches (the LDS-DMA small GEMM)
    c3b = torch.empty(B, H, D, device=dev, dtype=torch.bfloat16)
    if FUSED_QKV_ATTN and H <= 64 and hd == 20 and D % 8 == 0:
        # the Q|K|V projection inside the attention launch (the same MFMA products in the same k
        # order as the GEMM launch it replaces; qkv still written for the backward)
        c3, stats, q3 = ops.user_qkv_attention_fwd(xd, wb[:D3], bqkv, B, heads, hd, keep, c3b)
    else:
        qkv = torch.empty(BH, D3, device=dev, dtype=torch.float32)
        ops.small_gemm(ops.Gemm(xd, wb[:D3], qkv, BH, D3, D, D, D, D3, bias=bqkv))  # one N = 3D GEMM
        q3 = qkv.view(B, H, D3)
        c3, stats = ops.user_attention_fwd(q3, heads, hd, keep, c3b)
    e = torch.empty(BH, Qd, device=dev, dtype=torch.float32)
    ops.small_gemm(ops.Gemm(c3b, wb[D3:], e, BH, Qd, D, D, D, Qd, bias=b1, act=1), tile=RD_ATT_FC1)
    e3 = e.view(B, H, Qd)
    if not pool:  # the caller runs the pool fused with the scores (UserStepFn)
        return None, [q3, stats, c3, c3b, e3, None, wb, w2, xd, wbt]
    u, alpha = ops.additive_pool_fwd(c3, e3, w2, b2, keep)
    return u, [q3, stats, c3, c3b, e3, alpha, wb, w2, xd, wbt]


def _user_enc_bwd(saved, du, dx, B: int, H: int, heads: int, hd: int, drop, dev_off, keep, pre=None,
                  defer: bool = False):
    """Backward of :func:`_user_enc_fwd` for ``du [B, D]``: the input gradient goes into ``dx
    [B*H, D]`` (the dropout backward in the dgrad epilogue) -> the ten weight gradients."""
    q3, stats, c3, c3b, e3, alpha, wb, w2, xd, wbt = saved
    D = c3.shape[-1]
    BH, D3 = B * H, 3 * D
    Qd = wb.shape[0] - D3
    dev = c3.device
    # additive pool backward: dx_direct = alpha du, dpre = da w2 (1 - e^2); dw2 = e^T da and
    # db2 = sum da join the weight-gradient launch below (da as column 0 of [BH, 8]: a small-GEMM
    # desc with M = 8, db2 from its column sums) -- no partial rows, no colsum launches
    # The producers also round their outputs to bf16 where a GEMM only consumes them (the values
    # the GEMM's own fp32 loads rounded to): dpre for dctx += dpre W1 and dQ|dK|dV for the input
    # and Q|K|V weight gradients -- bf16 x bf16 launches run on the LDS-DMA small GEMM.  The
    # att_fc1 weight gradient keeps the fp32 dpre (its bias gradient is a near-cancelling column
    # sum: from bf16 terms it measured 6 % off the fp32 oracle)
    lib = ops.native.require_for(c3)
    da8 = None
    if pre is not None:  # the pool's backward ran fused with the forward (user_pool_score)
        dctx, dpre, dpre_b, da8 = pre
    elif H <= 64 and c3.dtype == torch.float32 and e3.dtype == torch.float32:
        dctx, dpre, da8, dpre_b = lib.upool_bwd_da(c3.contiguous(), e3.contiguous(), alpha.contiguous(),
                                                   w2.reshape(-1).float().contiguous(), du.float().contiguous(), True)
    else:
        dctx, dpre, dw2, db2 = ops.additive_pool_bwd(c3, e3, alpha, w2, du, True)
        dpre_b = dpre.to(torch.bfloat16)
    dpre2 = dpre.view(BH, Qd)
    if wbt is not None and FUSED_QKV_ATTN and H <= 64 and hd == 20:
        # dctx += dpre W1 inside the attention backward launch (on the k-contiguous W1^T [D, Qd])
        dqkv = ops.user_attention_bwd_dctx(q3, stats, dctx, dpre_b.view(BH, Qd), wbt, heads, hd, keep).view(BH, D3)
    else:
        if wbt is not None:  # += dpre W1 on W1^T: the register-direct GEMM
            ops.small_gemm(ops.Gemm(dpre_b.view(BH, Qd), wbt, dctx, BH, D, Qd, Qd, Qd, D, accumulate=True),
                           tile=RD_DCTX)
        else:
            ops.small_gemm(ops.Gemm(dpre_b.view(BH, Qd), wb[D3:], dctx, BH, D, Qd, Qd, D, D, b_mode=1,
                                    accumulate=True))  # += dpre W1
        dqkv = ops.user_attention_bwd(q3, stats, dctx, heads, hd, keep, True).view(BH, D3)
    p, seed, off = drop
    # dx = [dQ | dK | dV] [Wq; Wk; Wv] o Z: one GEMM with K = 3D over the bf16 weight stack,
    # the dropout backward in its epilogue
    ekw = dict(pdrop=p, drop_on=3, drop_ld=D, seed=seed, offset=off) if p > 0 else {}
    # (on a k-contiguous W^T the register-direct form measured slower here: 28.1 vs 26.5 us)
    dgrad = ops.Gemm(dqkv, wb[:D3], dx, BH, D, D3, D3, D, D, b_mode=1, **ekw)
    # weight gradients: [dWq; dWk; dWv] = [dQ|dK|dV]^T X' (one M = 3D GEMM; X' bf16) and dW1 =
    # dpre^T ctx (fp32 operands: the mixed-dtype kernel); the bias gradients (column sums of
    # dQ|dK|dV and dpre, fp32) come out of the same launch (asum).  The input gradient has no
    # dependence on them: all three share ONE launch (weight gradients on a side stream beside
    # the input gradient measured slower: profiles/r3_ab_side_score_wgrad.txt)
    gqkv = torch.empty(D3, D, device=dev)
    gw1 = torch.empty(Qd, D, device=dev)
    gbqkv = torch.empty(D3, device=dev)
    gb1 = torch.empty(Qd, device=dev)
    wg = (ops.Gemm(dqkv, xd, gqkv, D3, D, BH, D3, D, D, a_mode=1, b_mode=1, asum=gbqkv),
          ops.Gemm(dpre2, c3b.view(BH, D), gw1, Qd, D, BH, Qd, D, D, a_mode=1, b_mode=1, asum=gb1))
    if da8 is not None:
        dw2 = torch.empty(8, Qd, device=dev)
        db2 = torch.empty(8, device=dev)
        wg += (ops.Gemm(da8, e3.reshape(BH, Qd), dw2, 8, Qd, BH, 8, Qd, Qd, a_mode=1, b_mode=1, asum=db2),)
        dw2, db2 = dw2[0], db2[:1]
    if defer and dx.is_cuda:
        # the input gradient now (the news-gradient segment sum reads it next; bf16 x bf16: the
        # LDS-DMA ring, unsplit), the weight gradients on the side stream or held back for the
        # text fc's backward launch (an end-of-backward callback runs them when no such launch comes)
        ops.small_gemm(dgrad, dev_off=dev_off)
        _PENDING_GEMMS.clear()  # (left over only by a backward that raised: its tensors are gone)
        _PENDING_GEMMS.extend(wg)
        torch.autograd.Variable._execution_engine.queue_callback(_flush_pending_gemms)
    else:
        ops.small_gemm(dgrad, *wg, dev_off=dev_off)
    # every gradient returned as a fresh view: autograd keeps a returned gradient as .grad only
    # when nothing else references it and clones it otherwise -- a side-stream GEMM still holds
    # gw1 / gb1 (its output), and a clone now would copy them before that GEMM wrote them
    return (gqkv[:D], gbqkv[:D], gqkv[D:2 * D], gbqkv[D:2 * D], gqkv[2 * D:], gbqkv[2 * D:], gw1.view_as(gw1),
            gb1.view_as(gb1), dw2.view(1, -1), db2.view(1))


class UserStepFn(torch.autograd.Function):
    """``loss, scores = UserStepFn(v, inv, perm, ptr, ...)`` for news vectors ``v [U, D]``: the
    device user side of a training / validation step.

    ``inv [R]`` maps the batch's occurrences (``B*C`` candidates, then ``B*H`` history
    slots) to rows of ``v``; ``perm / ptr`` group them per news for the segment sum (+ LDP).
    The user encoder is :func:`_user_enc_fwd` / :func:`_user_enc_bwd`; ``meta[-1]`` is the
    mask_padding key mask (the batch's history ids, int32 [B, H], or None).  (Round 2 first
    applied the input-dropout mask inside every GEMM tile's operand loads; each of the ~21
    column tiles redid its rows' Philox draws.)"""

    @staticmethod
    def forward(ctx, v, inv, perm, ptr, wq, bq, wk, bk, wv, bv, w1, b1, w2, b2, meta):
        B, C, H, heads, hd, act, drop, dev_off, ldp, padded, keep, one, casts, grad_on = meta
        D = v.shape[1]
        BC = B * C
        # the pool, the scores / loss and the pool's backward in one launch (user_pool_score)
        # where its domain holds; the separate kernels otherwise
        fuse = v.is_cuda and H <= 64 and C <= 16 and 256 <= D <= 512 and D % 4 == 0
        u, saved = _user_enc_fwd(v, inv[BC:], (wq, bq, wk, bk, wv, bv, w1, b1, w2, b2), B, H, heads, hd, drop,
                                 dev_off, keep, casts, pool=not fuse)
        # per-occurrence news gradients: the candidate rows come straight from the scoring
        # kernel (candidates read from v by index: no gathered copy), the history rows from the
        # user encoder's dgrad in the backward
        rows = torch.empty(inv.numel(), D, device=v.device, dtype=torch.float32)
        tail = ()
        if fuse:
            c3, e3 = saved[2], saved[4]
            want_bwd = grad_on and any(ctx.needs_input_grad)  # (validation: forward only)
            loss, scores, *tail = ops.native.require_for(v).user_pool_score(
                c3, e3, w2.reshape(-1).float().contiguous(), b2.reshape(-1).float().contiguous(), keep, v,
                inv[:BC], 1 if act == "sigmoid" else 0, rows[:BC], want_bwd)
            if loss.numel() == 0:  # outside the fused kernel's domain after all
                fuse, tail = False, ()
                u, saved[5] = ops.additive_pool_fwd(c3, e3, w2, b2, keep)
            elif not want_bwd:
                tail = ()
            du = None
        if not fuse:
            loss, scores, du = ops.score_ce_rows(v, inv[:BC], u, act, rows[:BC])
        ctx.n_tail = len(tail)
        ctx.save_for_backward(v, inv, perm, ptr, rows, du, *saved, *tail)
        ctx.meta = meta
        ctx.mark_non_differentiable(scores)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the scores (one fill launch)
        return loss, scores

    @staticmethod
    def backward(ctx, gloss, gscores):
        v, inv, perm, ptr, rows, du, *saved = ctx.saved_tensors
        pre = None
        if ctx.n_tail:
            saved, pre = saved[:-ctx.n_tail], list(saved[-ctx.n_tail:])
        B, C, H, heads, hd, act, drop, dev_off, ldp, padded, keep, one, _, _ = ctx.meta
        BC = B * C
        if gloss is not one:  # the engine seeds the backward with its persistent ones tensor: no scale
            rows[:BC].mul_(gloss)
            if pre is not None:  # the fused tail's backward pieces are linear in the loss gradient
                for t in pre:
                    t.mul_(gloss)
            else:
                du = du * gloss
        grads = _user_enc_bwd(saved, du, rows[BC:], B, H, heads, hd, drop, dev_off, keep, pre, defer=True)
        clip, noise, lseed, loff = ldp
        # the noise offset's step part is the device counter (dev_off): graph replays draw fresh noise
        dv = ops.segment_sum_rows(rows, inv, v.shape[0], clip, noise, lseed, loff, seg=(perm, ptr), zero_empty=padded,
                                  dev_off=dev_off if noise > 0 else None)
        return (dv, None, None, None) + grads + (None,)


def user_step(v, inv, perm, ptr, user_encoder, B: int, C: int, H: int, act: str, drop, dev_off, ldp, padded: bool,
              keep=None, one=None, casts=None):
    """Device user side of a step (see :class:`UserStepFn`) -> ``(loss, scores)``.  ``keep``:
    the mask_padding key mask (history ids [B, H], nonzero = real slot) or None.  ``one``: the
    tensor the caller will seed ``loss.backward`` with when it is a ones tensor (the backward
    then skips the scale by the incoming gradient)."""
    mha, pool = user_encoder.multihead_attention, user_encoder.additive_attention
    if keep is not None:
        keep = keep.reshape(B, H)
        keep = keep if keep.dtype == torch.int32 and keep.is_contiguous() else keep.to(torch.int32).contiguous()
    meta = (B, C, H, mha.n_heads, mha.d_k, act, drop, dev_off, ldp, padded, keep, one, casts, torch.is_grad_enabled())
    return UserStepFn.apply(v, inv, perm, ptr, mha.W_Q.weight, mha.W_Q.bias, mha.W_K.weight, mha.W_K.bias,
                            mha.W_V.weight, mha.W_V.bias, pool.att_fc1.weight, pool.att_fc1.bias,
                            pool.att_fc2.weight, pool.att_fc2.bias, meta)


_ARANGE: dict = {}


class UserEncoderFn(torch.autograd.Function):
    """The user encoder as a module call on the device (``encoder.py:36-56``: input dropout ->
    MHSA -> additive pool): ``clicked [B, H, D] -> u [B, D]`` on the same kernels as the
    training step (:func:`_user_enc_fwd` / :func:`_user_enc_bwd`), with autograd for the
    clicked-news rows and the ten weights.  No vendor GEMM, no torch dropout."""

    @staticmethod
    def forward(ctx, clicked, wq, bq, wk, bk, wv, bv, w1, b1, w2, b2, meta):
        heads, hd, drop, keep = meta
        B, H, D = clicked.shape
        key = (B * H, clicked.device)
        if key not in _ARANGE:
            _ARANGE[key] = torch.arange(B * H, device=clicked.device, dtype=torch.int32)
        u, saved = _user_enc_fwd(clicked.reshape(B * H, D).float().contiguous(), _ARANGE[key],
                                 (wq, bq, wk, bk, wv, bv, w1, b1, w2, b2), B, H, heads, hd, drop, None, keep)
        ctx.save_for_backward(*saved)
        ctx.meta = meta
        ctx.shape = (B, H, D)
        return u

    @staticmethod
    def backward(ctx, du):
        heads, hd, drop, keep = ctx.meta
        B, H, D = ctx.shape
        dx = torch.empty(B * H, D, device=du.device, dtype=torch.float32)
        grads = _user_enc_bwd(list(ctx.saved_tensors), du.float().contiguous(), dx, B, H, heads, hd, drop, None, keep)
        return (dx.view(B, H, D),) + grads + (None,)


def user_encoder_device(user_encoder, clicked, keep=None):
    """``UserEncoder.forward`` on the device (see :class:`UserEncoderFn`).  Train-mode input
    dropout draws a Philox mask keyed by the module's ``drop_seed`` (config seed + client rank)
    and its per-call counter ``drop_calls`` (in the engine's checkpointed state)."""
    mha, pool = user_encoder.multihead_attention, user_encoder.additive_attention
    p = float(user_encoder.dropout_rate) if user_encoder.training else 0.0
    seed = int(getattr(user_encoder, "drop_seed", 0))
    drop = (p, seed, 0)
    if p > 0:
        user_encoder.drop_calls = int(getattr(user_encoder, "drop_calls", 0)) + 1
        drop = (p, seed, user_encoder.drop_calls)
    if keep is not None:
        keep = keep.to(torch.int32).contiguous()
    return UserEncoderFn.apply(clicked, mha.W_Q.weight, mha.W_Q.bias, mha.W_K.weight, mha.W_K.bias, mha.W_V.weight,
                               mha.W_V.bias, pool.att_fc1.weight, pool.att_fc1.bias, pool.att_fc2.weight,
                               pool.att_fc2.bias, (mha.n_heads, mha.d_k, drop, keep))


class HeadFCFn(torch.autograd.Function):
    """The text head's ``fc`` (``encoder.py:22,29``: [n, 768] -> [n, 400]) on the small MFMA
    GEMM: forward NT, backward dgrad (NN), wgrad (TN) in one launch, bias gradient by colsum."""

    @staticmethod
    def forward(ctx, x, w, b, xb=None, wb=None, wbt=None):
        """``xb`` / ``wb`` (optional): x and w already rounded to bf16 (the pool's second output,
        the step's cast launch) -- the GEMMs round their fp32 operands to bf16 on the way into LDS
        anyway, so the products are the same, at half the bytes and on the bf16 fast path."""
        n, K = x.shape
        N = w.shape[0]
        x = x.contiguous()
        xg = xb if xb is not None else x
        wg = wb if wb is not None else w
        y = torch.empty(n, N, device=x.device, dtype=torch.float32)
        ops.small_gemm(ops.Gemm(xg, wg, y, n, N, K, K, K, N, bias=b))
        ctx.save_for_backward(xg, wg, wbt)
        ctx.into = _slots(w, b) if ctx.needs_input_grad[1] and ctx.needs_input_grad[2] else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, _ = ctx.saved_tensors
        n, K = x.shape
        N = w.shape[0]
        dy = dy.contiguous().float()
        dx = torch.empty(n, K, device=x.device, dtype=torch.float32)

        if ctx.into is not None:  # into the flat gradient's slots (N > 1)
            (dw, db), pids = ctx.into
            _GRAD_WRITTEN.update(pids)
        else:
            dw = torch.empty(N, K, device=x.device, dtype=torch.float32)
            db = torch.empty(N, device=x.device, dtype=torch.float32)
        wgrad = ops.Gemm(dy, x, dw, N, K, n, N, K, K, a_mode=1, b_mode=1, asum=db)
        # dgrad, wgrad and the bias gradient (dy's column sums, from the wgrad's dy tiles) in one
        # launch -- with the user encoder's weight gradients when its backward held them back
        gs = (ops.Gemm(dy, w, dx, n, K, N, N, K, K, b_mode=1), wgrad, *take_pending_gemms(4))
        early = _AFTER_USER_WGRADS[0] if len(gs) > 2 else None
        if defer_active() and early is None:  # the weight gradients' split-K reduce rides in the head's reduce launch
            lib = ops.native.require_for(dy)
            lib.small_gemm_set_defer(True)
            _DEFERRED[0] = True
            try:
                ops.small_gemm(*gs)
            finally:
                lib.small_gemm_set_defer(False)
        else:
            ops.small_gemm(*gs)
        if early is not None:  # the user-encoder weight gradients are final here
            early()
        if ctx.into is not None:
            return dx, None, None, None, None, None
        return dx, dw.view_as(dw), db.view_as(db), None, None, None
