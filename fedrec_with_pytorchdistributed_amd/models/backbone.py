"""Transformer text backbone with DistilBERT's module tree (so the state_dict keys are the
reference's ``text_encoder.DistillBert.*`` keys) and a compute path built
on the engine's own ops instead of HF modules.

Reference: ``encoder.py:19,27`` -- ``DistilBertModel.from_pretrained(...)(tokens,
attention_mask=mask)[0]``; frozen at ``model.py:25-26``; 6 post-LN blocks (C26).

Compute layout (MI355X path):

* the fp32 ``nn.Parameter`` tensors stay the source of truth (state_dict round-trips a
  reference checkpoint bit-exactly);
* :meth:`compute_weights` packs them once into device-resident compute tensors: Q|K|V
  fused into one ``[3D, D]`` bf16 weight (one GEMM with N = 2304 instead of three),
  biases fp32.  The pack is cached and rebuilt only when the fp32 weights change
  (``invalidate()``: load_state_dict, optimizer step in unfrozen mode);
* :meth:`forward` runs ``embed_ln -> [qkv GEMM -> title attention -> out GEMM -> LN(+res)
  -> FFN1 GEMM(+GELU) -> FFN2 GEMM -> LN(+res)] x L`` through :mod:`..ops`.

Initialisation follows HF DistilBERT ``_init_weights`` (normal(0, 0.02) for linears and
embeddings, zero biases, LN = (1, 0), padding row 0 of the word table zeroed).  There are
no pretrained weights offline.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
from torch import nn

from ..config import BackboneConfig
from .. import ops


# the packed title path (one launch per layer op over the whole batch of titles, packed
# attention) for the device bf16 backbone; False only in the tests comparing it with the
# per-op path
TITLE_PACK = True

class _Embeddings(nn.Module):
    def __init__(self, c: BackboneConfig):
        super().__init__()
        self.word_embeddings = nn.Embedding(c.vocab_size, c.dim, padding_idx=0)
        self.position_embeddings = nn.Embedding(c.max_position, c.dim)
        self.LayerNorm = nn.LayerNorm(c.dim, eps=c.ln_eps)


class _Attention(nn.Module):
    def __init__(self, c: BackboneConfig):
        super().__init__()
        self.q_lin = nn.Linear(c.dim, c.dim)
        self.k_lin = nn.Linear(c.dim, c.dim)
        self.v_lin = nn.Linear(c.dim, c.dim)
        self.out_lin = nn.Linear(c.dim, c.dim)


class _FFN(nn.Module):
    def __init__(self, c: BackboneConfig):
        super().__init__()
        self.lin1 = nn.Linear(c.dim, c.hidden_dim)
        self.lin2 = nn.Linear(c.hidden_dim, c.dim)


class _Block(nn.Module):
    def __init__(self, c: BackboneConfig):
        super().__init__()
        self.attention = _Attention(c)
        self.sa_layer_norm = nn.LayerNorm(c.dim, eps=c.ln_eps)
        self.ffn = _FFN(c)
        self.output_layer_norm = nn.LayerNorm(c.dim, eps=c.ln_eps)


class _Transformer(nn.Module):
    def __init__(self, c: BackboneConfig):
        super().__init__()
        self.layer = nn.ModuleList([_Block(c) for _ in range(c.n_layers)])


class Backbone(nn.Module):
    """``DistillBert`` sub-module of the text encoder."""

    def __init__(self, c: BackboneConfig):
        super().__init__()
        self.cfg = c
        self.embeddings = _Embeddings(c)
        self.transformer = _Transformer(c)
        self._pack: Optional[Dict] = None
        self._pack_key = None
        self._stale = True
        self._cast_plan_t = None
        self.version = 0  # bumped whenever the weights may have changed (hidden-state caches key on it)
        # train-mode dropout: Philox key (the engine sets seed + rank) and a per-forward counter;
        # a forward's sites use offsets 1024 * call + {0: embeddings, 1 + 2l: attention of
        # layer l, 2 + 2l: FFN of layer l}, so the backward regenerates every mask
        self.drop_seed = 0
        self._drop_calls = 0
        self.reset_parameters()

    # -------------------------------------------------------------------------------
    @torch.no_grad()
    def reset_parameters(self) -> None:
        std = self.cfg.init_std
        for m in self.modules():
            if isinstance(m, nn.Linear):
                m.weight.normal_(0.0, std)
                m.bias.zero_()
            elif isinstance(m, nn.Embedding):
                m.weight.normal_(0.0, std)
                if m.padding_idx is not None:
                    m.weight[m.padding_idx].zero_()
            elif isinstance(m, nn.LayerNorm):
                m.weight.fill_(1.0)
                m.bias.zero_()
        self.invalidate()

    def invalidate(self) -> None:
        self._stale = True
        self.version += 1

    @torch.no_grad()
    def fingerprint(self) -> torch.Tensor:
        """A checksum of every weight (fp64 sum and sum of squares per tensor, on the host):
        identical weights give identical fingerprints (same deterministic reductions)."""
        parts = [torch.stack([p.detach().double().sum(), p.detach().double().square().sum()])
                 for p in self.parameters()]
        return torch.cat(parts).cpu() if parts else torch.zeros(0, dtype=torch.float64)

    def invalidate_if_changed(self, before: torch.Tensor) -> bool:
        """Invalidate (compute pack + hidden-state caches) only when the weights differ from
        the ``before`` fingerprint; a sync of a frozen backbone between bitwise-identical
        replicas (every client starts from the same seed / checkpoint, and a mean over a
        power-of-two client count is exact) then keeps the cache.  Returns True if invalidated."""
        if torch.equal(self.fingerprint(), before):
            return False
        self.invalidate()
        return True

    @property
    def pack_stale(self) -> bool:
        return self._pack is None or self._stale

    def _load_from_state_dict(self, *args, **kwargs):  # keep the compute pack coherent
        self.invalidate()
        return super()._load_from_state_dict(*args, **kwargs)

    @torch.no_grad()
    def compute_weights(self, dtype: torch.dtype) -> Dict:
        dev = self.embeddings.word_embeddings.weight.device
        key = (dtype, dev)
        if self._pack is not None and self._pack_key == key:
            if not self._stale:
                return self._pack
            # an optimizer step (or a load) changed the masters: refresh the existing compute
            # copies in place, all of them in one launch (csrc/adam.hip multi_cast) instead of
            # a cat + cast launch per weight
            lib = ops.native.lib() if dev.type == "cuda" else None
            if lib is not None and lib.multi_cast(*self._cast_plan) and (
                    self._cast_plan_t is None or lib.multi_cast_t(*self._cast_plan_t)):
                self._stale = False
                return self._pack
        e = self.embeddings
        pack: Dict = {
            "word": e.word_embeddings.weight.detach().to(dtype).contiguous(),
            "pos": e.position_embeddings.weight.detach().to(dtype).contiguous(),
            "emb_ln_w": e.LayerNorm.weight.detach().float().contiguous(),
            "emb_ln_b": e.LayerNorm.bias.detach().float().contiguous(),
            "layers": [],
        }
        for blk in self.transformer.layer:
            a = blk.attention
            pack["layers"].append({
                "wqkv": torch.cat([a.q_lin.weight, a.k_lin.weight, a.v_lin.weight], 0).to(dtype).contiguous(),
                "bqkv": torch.cat([a.q_lin.bias, a.k_lin.bias, a.v_lin.bias], 0).float().contiguous(),
                "wo": a.out_lin.weight.detach().to(dtype).contiguous(),
                "bo": a.out_lin.bias.detach().float().contiguous(),
                "ln1_w": blk.sa_layer_norm.weight.detach().float().contiguous(),
                "ln1_b": blk.sa_layer_norm.bias.detach().float().contiguous(),
                "w1": blk.ffn.lin1.weight.detach().to(dtype).contiguous(),
                "b1": blk.ffn.lin1.bias.detach().float().contiguous(),
                "w2": blk.ffn.lin2.weight.detach().to(dtype).contiguous(),
                "b2": blk.ffn.lin2.bias.detach().float().contiguous(),
                "ln2_w": blk.output_layer_norm.weight.detach().float().contiguous(),
                "ln2_b": blk.output_layer_norm.bias.detach().float().contiguous(),
            })
        # in-place refresh plan: every master whose compute copy is not the master itself
        src, dst = [e.word_embeddings.weight, e.position_embeddings.weight], [pack["word"], pack["pos"]]
        for blk, L in zip(self.transformer.layer, pack["layers"]):
            a = blk.attention
            D = a.q_lin.weight.shape[0]
            for i, lin in enumerate((a.q_lin, a.k_lin, a.v_lin)):
                src += [lin.weight, lin.bias]
                dst += [L["wqkv"][i * D:(i + 1) * D], L["bqkv"][i * D:(i + 1) * D]]
            src += [a.out_lin.weight, blk.ffn.lin1.weight, blk.ffn.lin2.weight]
            dst += [L["wo"], L["w1"], L["w2"]]
        self._cast_plan = ([t.detach() for t in src], dst)
        # unfrozen training: transposed bf16 copies for the input-gradient GEMMs (they run on
        # W^T), refreshed in the same step by one transposing launch (multi_cast_t) instead of
        # a `.t().contiguous()` copy per weight in every backward
        self._cast_plan_t = None
        if not self.cfg.frozen and dev.type == "cuda" and dtype == torch.bfloat16:
            srct, dstt = [], []
            for blk, L in zip(self.transformer.layer, pack["layers"]):
                a = blk.attention
                D = a.q_lin.weight.shape[0]
                L["wqkv_t"] = L["wqkv"].t().contiguous()
                L["wo_t"] = L["wo"].t().contiguous()
                L["w1_t"] = L["w1"].t().contiguous()
                L["w2_t"] = L["w2"].t().contiguous()
                for i, lin in enumerate((a.q_lin, a.k_lin, a.v_lin)):
                    srct.append(lin.weight)
                    dstt.append(L["wqkv_t"][:, i * D:(i + 1) * D])
                srct += [a.out_lin.weight, blk.ffn.lin1.weight, blk.ffn.lin2.weight]
                dstt += [L["wo_t"], L["w1_t"], L["w2_t"]]
            self._cast_plan_t = ([t.detach() for t in srct], dstt)
        self._pack, self._pack_key, self._stale = pack, key, False
        return pack

    # -------------------------------------------------------------------------------
    def dropout_sites(self):
        """Per-forward dropout sites ``(embed, [(attn_l, ffn_l)])``, each ``(p, seed, offset)`` or
        None (p = 0)."""
        c = self.cfg
        base = self._drop_calls * 1024
        self._drop_calls += 1

        def site(p, k):
            return (float(p), int(self.drop_seed), base + k) if p > 0 else None

        return site(c.dropout, 0), [(site(c.attention_dropout, 1 + 2 * i), site(c.dropout, 2 + 2 * i))
                                    for i in range(c.n_layers)]

    @torch.no_grad()
    def forward(self, tokens: torch.Tensor, mask: torch.Tensor, dtype: torch.dtype, dropout: bool = False,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``tokens, mask [n, T]`` -> last hidden state ``[n*T, D]`` in ``dtype`` (eval mode;
        ``dropout`` = HF train-mode dropout, used by the reference-compat replay Q4).  ``out``
        (packed device path): the last LayerNorm writes straight into it (e.g. the hidden-state
        cache's rows); other paths copy into it."""
        c = self.cfg
        P = self.compute_weights(dtype)
        if dropout:
            return _into(self._forward_dropout(tokens, mask, P), out)
        if (tokens.is_cuda and dtype == torch.bfloat16 and c.dim % 256 == 0 and c.n_layers > 0
                and tokens.shape[1] <= 64 and TITLE_PACK):
            return self._forward_packed(tokens, mask, P, out)
        x = ops.embed_ln(tokens, P["word"], P["pos"], P["emb_ln_w"], P["emb_ln_b"], c.ln_eps, dtype)
        for L in P["layers"]:
            qkv = ops.linear(x, L["wqkv"], L["bqkv"], out_dtype=dtype)
            ctx = ops.title_attention(qkv, mask, c.n_heads)
            # residual adds ride in the LayerNorm kernel (LN(h + x)): a residual read in the GEMM
            # epilogue stalls the ping-pong schedule (out-proj 638 -> 850 TF without it)
            h = ops.linear(ctx, L["wo"], L["bo"], out_dtype=dtype)
            x = ops.layer_norm(h, L["ln1_w"], L["ln1_b"], c.ln_eps, dtype, residual=x)
            f = ops.linear(x, L["w1"], L["b1"], act="gelu", out_dtype=dtype)
            h = ops.linear(f, L["w2"], L["b2"], out_dtype=dtype)
            x = ops.layer_norm(h, L["ln2_w"], L["ln2_b"], c.ln_eps, dtype, residual=x)
        return _into(x, out)

    def _forward_dropout(self, tokens: torch.Tensor, mask: torch.Tensor, P: Dict) -> torch.Tensor:
        """Train-mode forward without gradients (frozen backbone, Q4 replay): the unpacked
        path with HF DistilBERT's three dropout sites (csrc/dropout.hip, title_attn.hip)."""
        c = self.cfg
        emb, layers = self.dropout_sites()
        x = ops.embed_ln(tokens, P["word"], P["pos"], P["emb_ln_w"], P["emb_ln_b"], c.ln_eps, P["word"].dtype)
        if emb is not None:
            x = ops.dropout_add(x, None, *emb)
        for L, (sa, sf) in zip(P["layers"], layers):
            qkv = ops.linear(x, L["wqkv"], L["bqkv"])
            ctx = ops.title_attention(qkv, mask, c.n_heads, sa)
            h = ops.linear(ctx, L["wo"], L["bo"])
            x = ops.layer_norm(h, L["ln1_w"], L["ln1_b"], c.ln_eps, residual=x)
            f = ops.linear(x, L["w1"], L["b1"], act="gelu")
            h = ops.linear(f, L["w2"], L["b2"])
            if sf is not None:
                x = ops.layer_norm(ops.dropout_add(h, x, *sf), L["ln2_w"], L["ln2_b"], c.ln_eps)
            else:
                x = ops.layer_norm(h, L["ln2_w"], L["ln2_b"], c.ln_eps, residual=x)
        return x

    def _forward_packed(self, tokens: torch.Tensor, mask: torch.Tensor, P: Dict,
                        out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The same forward over the packed row order of ``ops.title_plan``: the rows read as
        keys/values (real tokens) come first, so the fused QKV GEMM skips the K and V columns
        of every padding row (~2/3 of MIND title rows) and the attention skips key tiles past
        each title's length.  All other ops are row-wise; the last LayerNorm stores rows back
        in title order, so the output is identical in layout (and, up to fp32 summation
        order, in value) to the unpacked path.

        (Splitting the titles over two streams interleaved layer by layer measured no gain:
        profiles/r1/bench_r1_backbone_streams_ab.jsonl.)"""
        holder = [None]
        for _ in self._packed_stages(tokens, mask, P, holder, 0, out):
            pass
        return holder[0]

    def _packed_stages(self, tokens: torch.Tensor, mask: torch.Tensor, P: Dict, holder: list, slot: int,
                       out: Optional[torch.Tensor] = None):
        """Generator: one ``yield`` per transformer layer."""
        c = self.cfg
        rowmap, src, kv_start, kv_len, qstart, n_kv = ops.title_plan(mask)
        x = ops.embed_ln_rows(tokens, src, P["word"], P["pos"], P["emb_ln_w"], P["emb_ln_b"], c.ln_eps)
        last = len(P["layers"]) - 1
        for li, L in enumerate(P["layers"]):
            qkv = ops.linear_split(x, L["wqkv"], L["bqkv"], n_kv, c.dim)
            ctx = ops.title_attention_packed(qkv, rowmap, kv_start, kv_len, qstart, c.n_heads)
            h = ops.linear(ctx, L["wo"], L["bo"])
            x = ops.layer_norm(h, L["ln1_w"], L["ln1_b"], c.ln_eps, residual=x)
            f = ops.linear(x, L["w1"], L["b1"], act="gelu")
            h = ops.linear(f, L["w2"], L["b2"])
            if li == last:
                x = ops.layer_norm_scatter(h, L["ln2_w"], L["ln2_b"], c.ln_eps, x, src, out)
            else:
                x = ops.layer_norm(h, L["ln2_w"], L["ln2_b"], c.ln_eps, residual=x)
            yield li
        holder[slot] = x

    def forward_train(self, tokens: torch.Tensor, mask: torch.Tensor, dtype: torch.dtype,
                      dropout: bool = False) -> torch.Tensor:
        """Differentiable forward for an unfrozen backbone (BASELINE config 5); ``dropout`` =
        HF train mode (embedding / attention-probability / FFN dropout with Philox counter
        masks that the backward regenerates).  Device: our kernels + their backward kernels
        through autograd Functions whose gradients land in the fp32 master parameters; host:
        the oracle ops (same masks, bit for bit) under plain autograd."""
        from ..ops import functional as OF
        from ..ops import reference as R

        c = self.cfg
        e = self.embeddings
        emb, sites = self.dropout_sites() if dropout else (None, [(None, None)] * c.n_layers)
        if not tokens.is_cuda or dtype != torch.bfloat16:
            x = R.embed_ln(tokens, e.word_embeddings.weight, e.position_embeddings.weight, e.LayerNorm.weight,
                           e.LayerNorm.bias, c.ln_eps)
            if emb is not None:
                x = R.dropout_add(x, None, *emb)
            for blk, (sa, sf) in zip(self.transformer.layer, sites):
                a = blk.attention
                wqkv = torch.cat([a.q_lin.weight, a.k_lin.weight, a.v_lin.weight], 0)
                bqkv = torch.cat([a.q_lin.bias, a.k_lin.bias, a.v_lin.bias], 0)
                qkv = R.linear(x, wqkv, bqkv)
                ctx = R.title_attention(qkv, mask, c.n_heads, sa)
                x = R.layer_norm(R.linear(ctx, a.out_lin.weight, a.out_lin.bias, residual=x),
                                 blk.sa_layer_norm.weight, blk.sa_layer_norm.bias, c.ln_eps)
                f = R.linear(x, blk.ffn.lin1.weight, blk.ffn.lin1.bias, act="gelu")
                if sf is not None:
                    h = R.dropout_add(R.linear(f, blk.ffn.lin2.weight, blk.ffn.lin2.bias), x, *sf)
                else:
                    h = R.linear(f, blk.ffn.lin2.weight, blk.ffn.lin2.bias, residual=x)
                x = R.layer_norm(h, blk.output_layer_norm.weight, blk.output_layer_norm.bias, c.ln_eps)
            return x
        P = self.compute_weights(dtype)
        x = OF.EmbedLNFn.apply(tokens.contiguous(), e.word_embeddings.weight, e.position_embeddings.weight,
                               e.LayerNorm.weight, e.LayerNorm.bias, c.ln_eps, P["word"], P["pos"])
        if emb is not None:
            x = OF.DropoutFn.apply(x, *emb)
        for blk, L, (sa, sf) in zip(self.transformer.layer, P["layers"], sites):
            a = blk.attention
            # fused block Functions; box: each LN backward hands its dx column sums (the bias grad
            # of the block half feeding it) to that block's backward, which runs next
            box1, box2 = {}, {}
            h = OF.AttnBlockFn.apply(x, a.q_lin.weight, a.k_lin.weight, a.v_lin.weight, a.q_lin.bias,
                                     a.k_lin.bias, a.v_lin.bias, a.out_lin.weight, a.out_lin.bias,
                                     mask.contiguous(), c.n_heads, L["wqkv"], L["bqkv"], L["wo"], box1, sa,
                                     (L.get("wqkv_t"), L.get("wo_t")))
            x = OF.LayerNormFn.apply(h, blk.sa_layer_norm.weight, blk.sa_layer_norm.bias, c.ln_eps, box1)
            h = OF.MLPBlockFn.apply(x, blk.ffn.lin1.weight, blk.ffn.lin1.bias, blk.ffn.lin2.weight,
                                    blk.ffn.lin2.bias, L["w1"], L["w2"], box2, sf, (L.get("w1_t"), L.get("w2_t")))
            x = OF.LayerNormFn.apply(h, blk.output_layer_norm.weight, blk.output_layer_norm.bias, c.ln_eps, box2)
        return x

    def hf_state_dict(self) -> Dict[str, torch.Tensor]:
        """Keys as HF ``DistilBertModel`` names them (for parity tests)."""
        return {k: v for k, v in self.state_dict().items()}


def _into(x: torch.Tensor, out: Optional[torch.Tensor]) -> torch.Tensor:
    if out is None:
        return x
    out.view_as(x).copy_(x)
    return out


def param_names(c: BackboneConfig) -> List[str]:
    names = ["embeddings.word_embeddings.weight", "embeddings.position_embeddings.weight",
             "embeddings.LayerNorm.weight", "embeddings.LayerNorm.bias"]
    for i in range(c.n_layers):
        p = f"transformer.layer.{i}."
        for m in ("attention.q_lin", "attention.k_lin", "attention.v_lin", "attention.out_lin"):
            names += [p + m + ".weight", p + m + ".bias"]
        names += [p + "sa_layer_norm.weight", p + "sa_layer_norm.bias"]
        for m in ("ffn.lin1", "ffn.lin2"):
            names += [p + m + ".weight", p + m + ".bias"]
        names += [p + "output_layer_norm.weight", p + "output_layer_norm.bias"]
    return names
