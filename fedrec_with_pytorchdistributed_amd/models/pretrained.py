"""Pretrained text-backbone weights from a LOCAL Hugging Face checkpoint.

The reference builds its text encoder with ``DistilBertModel.from_pretrained(
"distilbert-base-uncased")`` (``encoder.py:19``), i.e. it downloads pretrained weights.  This
framework never touches the network: ``--backbone.pretrained=PATH`` points at a local
directory written by ``save_pretrained`` (``config.json`` + ``model.safetensors`` /
``pytorch_model.bin``, sharded index files included) or at a single weights file, and the
weights are mapped onto :class:`~.backbone.Backbone`'s DistilBERT module tree.

* DistilBERT (``DistilBertModel`` / ``DistilBertForMaskedLM`` ...): keys map 1:1 after the
  ``distilbert.`` prefix is stripped; heads (``vocab_*``, classifiers) are ignored.
* BERT (BASELINE config 5's BERT-base): ``encoder.layer.i.attention.self.{query,key,value}``
  -> ``transformer.layer.i.attention.{q,k,v}_lin`` etc.; the token-type embedding row 0 is
  folded into the position table (every token has type 0 here), which is exact.

Loading is safe by construction: safetensors, or ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import json
import os
import re
from typing import Dict, Optional, Tuple

import torch

from ..config import BackboneConfig

_WEIGHT_FILES = ("model.safetensors", "pytorch_model.bin")
_INDEX_FILES = ("model.safetensors.index.json", "pytorch_model.bin.index.json")


def _load_file(path: str) -> Dict[str, torch.Tensor]:
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file

        return load_file(path, device="cpu")
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    return sd


def read_checkpoint(path: str) -> Tuple[Optional[dict], Dict[str, torch.Tensor]]:
    """-> ``(config.json dict or None, flat state dict)`` of a local HF checkpoint."""
    if os.path.isfile(path):
        return None, _load_file(path)
    if not os.path.isdir(path):
        raise FileNotFoundError(f"pretrained backbone: {path!r} is neither a file nor a directory")
    cfg = None
    cp = os.path.join(path, "config.json")
    if os.path.exists(cp):
        with open(cp) as f:
            cfg = json.load(f)
    for idx in _INDEX_FILES:
        ip = os.path.join(path, idx)
        if os.path.exists(ip):
            with open(ip) as f:
                shards = sorted(set(json.load(f)["weight_map"].values()))
            sd: Dict[str, torch.Tensor] = {}
            for s in shards:
                sd.update(_load_file(os.path.join(path, s)))
            return cfg, sd
    for w in _WEIGHT_FILES:
        wp = os.path.join(path, w)
        if os.path.exists(wp):
            return cfg, _load_file(wp)
    raise FileNotFoundError(f"pretrained backbone: no {' / '.join(_WEIGHT_FILES)} in {path!r}")


def config_from_hf(hf: dict, base: Optional[BackboneConfig] = None) -> BackboneConfig:
    """``config.json`` -> :class:`BackboneConfig` (frozen flag and name kept from ``base``)."""
    base = base or BackboneConfig()
    mt = hf.get("model_type", "distilbert")
    if mt == "distilbert":
        act = hf.get("activation", "gelu")
        c = BackboneConfig(name=base.name, vocab_size=hf["vocab_size"], dim=hf["dim"], n_layers=hf["n_layers"],
                           n_heads=hf["n_heads"], hidden_dim=hf["hidden_dim"],
                           max_position=hf["max_position_embeddings"], ln_eps=1e-12, frozen=base.frozen)
    elif mt == "bert":
        act = hf.get("hidden_act", "gelu")
        if hf.get("position_embedding_type", "absolute") != "absolute":
            raise ValueError("pretrained backbone: only absolute position embeddings are supported")
        c = BackboneConfig(name=base.name, vocab_size=hf["vocab_size"], dim=hf["hidden_size"],
                           n_layers=hf["num_hidden_layers"], n_heads=hf["num_attention_heads"],
                           hidden_dim=hf["intermediate_size"], max_position=hf["max_position_embeddings"],
                           ln_eps=hf.get("layer_norm_eps", 1e-12), frozen=base.frozen)
    else:
        raise ValueError(f"pretrained backbone: model_type {mt!r} (supported: distilbert, bert)")
    if act != "gelu":
        raise ValueError(f"pretrained backbone: activation {act!r} (the kernels implement erf GELU)")
    return c


_BERT_LAYER = [
    ("attention.self.query", "attention.q_lin"), ("attention.self.key", "attention.k_lin"),
    ("attention.self.value", "attention.v_lin"), ("attention.output.dense", "attention.out_lin"),
    ("attention.output.LayerNorm", "sa_layer_norm"), ("intermediate.dense", "ffn.lin1"),
    ("output.dense", "ffn.lin2"), ("output.LayerNorm", "output_layer_norm"),
]


def _ln_key(k: str) -> str:  # old TF-converted checkpoints name LayerNorm params gamma / beta
    return re.sub(r"LayerNorm\.gamma$", "LayerNorm.weight", re.sub(r"LayerNorm\.beta$", "LayerNorm.bias", k))


def convert_state_dict(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """HF DistilBERT / BERT keys -> :class:`~.backbone.Backbone` keys (heads dropped)."""
    sd = {_ln_key(k): v for k, v in sd.items()}
    is_bert = any(".attention.self.query." in k for k in sd)
    out: Dict[str, torch.Tensor] = {}
    for k, v in sd.items():
        for p in ("distilbert.", "bert.", "model."):
            if k.startswith(p):
                k = k[len(p):]
                break
        if not is_bert:
            if k.startswith("embeddings.") or k.startswith("transformer.layer."):
                out[k] = v
            continue
        if k in ("embeddings.word_embeddings.weight", "embeddings.position_embeddings.weight",
                 "embeddings.LayerNorm.weight", "embeddings.LayerNorm.bias"):
            out[k] = v
            continue
        m = re.match(r"encoder\.layer\.(\d+)\.(.+)\.(weight|bias)$", k)
        if m:
            i, mod, kind = m.groups()
            for src, dst in _BERT_LAYER:
                if mod == src:
                    out[f"transformer.layer.{i}.{dst}.{kind}"] = v
    if is_bert:
        tt = next((v for k, v in sd.items() if k.endswith("embeddings.token_type_embeddings.weight")), None)
        if tt is not None and "embeddings.position_embeddings.weight" in out:
            # BERT embeds word + position + token_type; all tokens are type 0 here
            out["embeddings.position_embeddings.weight"] = out["embeddings.position_embeddings.weight"] + tt[0]
    return out


@torch.no_grad()
def load_pretrained_backbone(backbone, path: str) -> Dict[str, list]:
    """Copy a local HF checkpoint into ``backbone`` (shapes must match its config).
    Returns ``{"missing": [...], "ignored": [...]}``; raises if any backbone key is missing."""
    hf_cfg, raw = read_checkpoint(path)
    if hf_cfg is not None:
        want = config_from_hf(hf_cfg, backbone.cfg)
        have = backbone.cfg
        for f in ("vocab_size", "dim", "n_layers", "n_heads", "hidden_dim", "max_position"):
            if getattr(want, f) != getattr(have, f):
                raise ValueError(f"pretrained backbone {path!r}: {f} = {getattr(want, f)} but the configured "
                                 f"backbone has {getattr(have, f)} (set --backbone.* to match)")
    sd = convert_state_dict(raw)
    own = backbone.state_dict()
    missing = [k for k in own if k not in sd]
    if missing:
        raise KeyError(f"pretrained backbone {path!r}: missing {len(missing)} tensors, e.g. {missing[:4]}")
    for k, t in own.items():
        if tuple(sd[k].shape) != tuple(t.shape):
            raise ValueError(f"pretrained backbone {path!r}: {k} has shape {tuple(sd[k].shape)}, "
                             f"expected {tuple(t.shape)}")
        t.copy_(sd[k].to(t.dtype))
    backbone.invalidate()
    return {"missing": [], "ignored": sorted(set(raw) - set(own))[:50]}
