"""Text encoder (backbone + additive-attention head + FC 400) and user encoder.

Module trees mirror the reference so state_dict keys match:

* ``TextEncoder``  (``encoder.py:12-30``): ``DistillBert`` / ``additive_attention``
  (``att_fc1 [384,768]``, ``att_fc2 [1,384]``) / ``fc [400,768]``.
* ``UserEncoder``  (``encoder.py:36-56``): ``multihead_attention`` (``W_Q, W_K, W_V``
  ``[400,400]``, Xavier-uniform weights, ``attention.py:64-67``; no output projection) /
  ``additive_attention`` (``att_fc1 [200,400]``, ``att_fc2 [1,200]``).

The text encoder is split into :meth:`TextEncoder.hidden` (frozen backbone, no grad,
bf16 on the device) and :meth:`TextEncoder.head` (trainable), which is what lets the
engine dedup titles, cache hidden states, and run the head VJP without re-running the
backbone.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from ..config import FedRecConfig
from ..ops import functional as OF
from .backbone import Backbone


class AdditiveAttention(nn.Module):
    """``attention.py:8-26``; the reference pools without a padding mask (Q7), ``keep`` is the
    mask_padding option."""

    def __init__(self, d_h: int, hidden_size: int = 200):
        super().__init__()
        self.att_fc1 = nn.Linear(d_h, hidden_size)
        self.att_fc2 = nn.Linear(hidden_size, 1)

    def forward(self, x: torch.Tensor, keep: torch.Tensor | None = None) -> torch.Tensor:
        return OF.additive_pool(x, self.att_fc1, self.att_fc2, keep)  # keep: mask_padding (Q7 option)


class MultiHeadAttention(nn.Module):
    """``attention.py:50-82`` (no output projection; the reference passes no mask, ``keep`` is
    the mask_padding option)."""

    def __init__(self, d_model: int, n_heads: int, d_k: int, d_v: int):
        super().__init__()
        assert d_k == d_v
        self.n_heads, self.d_k = n_heads, d_k
        self.W_Q = nn.Linear(d_model, d_k * n_heads)
        self.W_K = nn.Linear(d_model, d_k * n_heads)
        self.W_V = nn.Linear(d_model, d_v * n_heads)
        for m in (self.W_Q, self.W_K, self.W_V):
            nn.init.xavier_uniform_(m.weight, gain=1)

    def forward(self, x: torch.Tensor, keep: torch.Tensor | None = None) -> torch.Tensor:
        w = torch.cat([self.W_Q.weight, self.W_K.weight, self.W_V.weight], 0)
        b = torch.cat([self.W_Q.bias, self.W_K.bias, self.W_V.bias], 0)
        if x.is_cuda:  # one [B*H, 400] x [400, 1200] GEMM on the small MFMA kernel
            B, H, D = x.shape
            qkv = OF.HeadFCFn.apply(x.reshape(B * H, D).float(), w, b).view(B, H, -1)
        else:
            qkv = F.linear(x, w, b)
        # keep: mask_padding (Q7 option), the attention.py:76-78 key mask
        return OF.user_attention(qkv, self.n_heads, self.d_k, keep)


class UserEncoder(nn.Module):
    def __init__(self, cfg: FedRecConfig):
        super().__init__()
        self.dropout_rate = cfg.user_dropout
        # device path's train-mode input dropout: Philox key (the engine sets it from the config
        # seed and the client rank) and a per-forward counter (checkpointed via engine.state())
        self.drop_seed = (int(cfg.seed) << 20) + 2
        self.drop_calls = 0
        self.multihead_attention = MultiHeadAttention(cfg.news_dim, cfg.user_heads, cfg.user_head_dim,
                                                      cfg.user_head_dim)
        self.additive_attention = AdditiveAttention(cfg.news_dim, cfg.user_query_dim)
        self.mask_padding = cfg.mask_padding

    def forward(self, clicked: torch.Tensor, his_ids: torch.Tensor | None = None) -> torch.Tensor:
        """``clicked [B,H,400]``; ``his_ids [B,H]`` (0 = padding) masks the padded history
        slots when ``mask_padding`` is on (the reference attends over them: Q7)."""
        keep = (his_ids != 0) if (self.mask_padding and his_ids is not None) else None
        mha = self.multihead_attention
        if clicked.is_cuda and mha.n_heads * mha.d_k == clicked.shape[-1]:
            # the training step's kernels (Philox input dropout, small GEMMs, MHSA, pool)
            return OF.user_encoder_device(self, clicked, keep)
        x = F.dropout(clicked, p=self.dropout_rate, training=self.training)  # host path
        y = mha(x, keep)
        return self.additive_attention(y, keep)


class TextEncoder(nn.Module):
    def __init__(self, cfg: FedRecConfig):
        super().__init__()
        self.cfg = cfg
        self.DistillBert = Backbone(cfg.backbone)
        if cfg.backbone.pretrained:  # encoder.py:19 from_pretrained, from a LOCAL checkpoint
            from .pretrained import load_pretrained_backbone

            load_pretrained_backbone(self.DistillBert, cfg.backbone.pretrained)
        d = cfg.backbone.dim
        self.additive_attention = AdditiveAttention(d, cfg.text_query_dim or d // 2)
        self.fc = nn.Linear(d, cfg.news_dim)

    @property
    def compute_dtype(self) -> torch.dtype:
        dev = self.fc.weight.device
        if dev.type == "cuda" and self.cfg.precision == "bf16":
            return torch.bfloat16
        return torch.float32

    def hidden(self, text: torch.Tensor, dropout: bool | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
        """``text [n,2,T]`` -> last hidden state ``[n,T,D]``: no-grad inference for the frozen
        backbone (the reference, model.py:25-26); a differentiable forward when unfrozen.

        ``dropout``: HF train-mode dropout in the backbone.  None = on for the unfrozen
        backbone's training forward in train mode; the frozen backbone's news vectors are
        eval-mode as in ``gen_news_vecs`` (model.py:42) unless the caller asks for it (the
        reference's train-mode replay, model.py:73 -- Q4).  ``out`` (no-grad paths): the result
        is written there (the packed device forward stores its last LayerNorm into it)."""
        n, _, T = text.shape
        bb = self.DistillBert
        train = not bb.cfg.frozen and torch.is_grad_enabled()
        if dropout is None:
            dropout = train and self.training
        if train:
            h = bb.forward_train(text[:, 0, :].contiguous(), text[:, 1, :].contiguous(), self.compute_dtype, dropout)
        else:
            h = bb(text[:, 0, :], text[:, 1, :], self.compute_dtype, dropout=dropout, out=out)
        return h.view(n, T, -1)

    def fused_head_ok(self, title_len: int) -> bool:
        """The fused text-head kernels (``OF.TextHeadFn``) apply: device, bf16, supported shape."""
        if self.compute_dtype != torch.bfloat16:
            return False
        key = int(title_len)
        cache = self.__dict__.setdefault("_fused_ok", {})
        if key not in cache:
            cache[key] = OF.fused_head_supported(self.cfg.backbone.dim, self.additive_attention.att_fc1.out_features,
                                                 title_len)
        return cache[key]

    def head_rows(self, table: torch.Tensor, ids: torch.Tensor | None, title_len: int,
                  tokens: torch.Tensor | None = None, nreal: torch.Tensor | None = None,
                  w1b: torch.Tensor | None = None, fcb: torch.Tensor | None = None) -> torch.Tensor:
        """Trainable head over GATHERED hidden states: ``table [rows, D]`` bf16 (the HBM cache as
        rows), titles ``ids [U]`` (None: 0..U-1), ``title_len`` tokens each -> ``[U, 400]`` fp32.
        ``tokens [N, 2, T]`` int32 masks padding tokens when ``mask_padding`` is on (Q7).
        ``nreal`` (device int32 [1]): titles past it are padding (pooled = 0, no gradient).
        ``w1b`` / ``fcb``: att_fc1's / fc's weight already cast to bf16 this step (one cast launch
        per step; ``fcb`` may be the pair (fc, fc^T)); with ``fcb`` the pool also emits its rows in
        bf16 for the fc GEMMs."""
        aa = self.additive_attention
        tok = tokens if self.cfg.mask_padding else None
        pooled, pooled_b = OF.TextHeadFn.apply(aa.att_fc1.weight, aa.att_fc1.bias, aa.att_fc2.weight,
                                               aa.att_fc2.bias, table, ids, int(title_len), tok, nreal, w1b,
                                               fcb is not None)
        if fcb is None:
            return OF.HeadFCFn.apply(pooled, self.fc.weight, self.fc.bias)
        fcb, fcbt = fcb if isinstance(fcb, tuple) else (fcb, None)
        return OF.HeadFCFn.apply(pooled, self.fc.weight, self.fc.bias, pooled_b, fcb, fcbt)

    def head(self, hidden: torch.Tensor, token_mask: torch.Tensor | None = None) -> torch.Tensor:
        """Trainable head: ``[n,T,D] -> [n,400]`` (fp32).  ``token_mask [n,T]`` excludes padding
        tokens from the pooling when ``mask_padding`` is on (the reference pools over them: Q7)."""
        n, T, D = hidden.shape
        if hidden.is_cuda and not hidden.requires_grad and self.fused_head_ok(T):
            tokens = None
            if self.cfg.mask_padding and token_mask is not None:
                m = token_mask.to(torch.int32)
                tokens = torch.stack([m, m], 1).contiguous()
            return self.head_rows(hidden.reshape(n * T, D).contiguous(), None, T, tokens)
        keep = (token_mask != 0) if (self.cfg.mask_padding and token_mask is not None) else None
        pooled = self.additive_attention(hidden, keep)
        if pooled.is_cuda:  # K07 on the small MFMA GEMM (fwd + bwd), not the vendor library
            return OF.HeadFCFn.apply(pooled, self.fc.weight, self.fc.bias)
        return F.linear(pooled, self.fc.weight, self.fc.bias)

    def forward(self, text: torch.Tensor) -> torch.Tensor:
        return self.head(self.hidden(text), text[:, 1, :])
