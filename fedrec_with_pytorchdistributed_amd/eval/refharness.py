"""Run the reference's own Python model code side by side with this engine.

The reference (``/root/reference``) is a flat directory of modules that import each other
by bare name (``from encoder import ...``) and need three packages that are absent offline:
``pickle5`` (aliased to ``pickle``, as the survey's scratch runs did), ``wandb`` and
``opacus`` (no-op stubs: the harness never reaches the code that uses them).  Its
``TextEncoder`` calls ``DistilBertModel.from_pretrained("distilbert-base-uncased")``
(``encoder.py:19``); with no network or HF cache the harness builds a random-init
``DistilBertModel`` from a ``DistilBertConfig`` instead (eager attention, the survey's E-runs
did the same), whose weights are then overwritten with ours via ``load_state_dict``.

Only source files are imported -- nothing prebuilt or serialized from the reference is
loaded by this module.  The shipped ``UserData`` shard is read with the engine's own
non-executing loader (:mod:`..data.safe_pickle`).

Used by ``tests/test_reference_parity.py`` (loss / score / gradient parity on the shipped
shard) and ``benchmarks/ref_auc_ab.py`` (the reference's training loop vs ours on one
synthetic shard).
"""
from __future__ import annotations

import contextlib
import importlib
import os
import pickle
import sys
import types
from dataclasses import dataclass
from typing import Any, Dict, Iterator, Optional

REFERENCE_PATH = os.environ.get("FEDREC_REFERENCE", "/root/reference")
_MODULES = ("attention", "encoder", "dataset", "model", "evaluation_functions", "client")


def available(path: str = REFERENCE_PATH) -> bool:
    try:
        import transformers  # noqa: F401
    except Exception:
        return False
    return all(os.path.exists(os.path.join(path, f"{m}.py")) for m in ("attention", "encoder", "model", "dataset"))


def _stub_modules() -> Dict[str, types.ModuleType]:
    import importlib.machinery

    wandb = types.ModuleType("wandb")
    wandb.__spec__ = importlib.machinery.ModuleSpec("wandb", None)
    for f in ("login", "init", "log", "finish"):
        setattr(wandb, f, lambda *a, **k: None)
    opacus = types.ModuleType("opacus")
    opacus.__spec__ = importlib.machinery.ModuleSpec("opacus", None)

    class PrivacyEngine:  # client.py:270-281 only; never called by the harness
        def __init__(self, *a, **k):
            raise RuntimeError("opacus is not available offline (reference client.py:270)")

    opacus.PrivacyEngine = PrivacyEngine
    return {"pickle5": pickle, "wandb": wandb, "opacus": opacus}


@dataclass
class Reference:
    attention: Any
    encoder: Any
    dataset: Any
    model: Any
    client: Optional[Any]


def load(path: str = REFERENCE_PATH, with_client: bool = True) -> Reference:
    """Import the reference modules in isolation: afterwards ``sys.modules`` and ``sys.path``
    hold exactly what they held before (the bare names ``model`` / ``dataset`` would shadow
    other packages)."""
    saved = {m: sys.modules.pop(m) for m in list(_MODULES) + list(_stub_modules()) if m in sys.modules}
    stubs = _stub_modules()
    sys.modules.update(stubs)
    sys.path.insert(0, path)
    try:
        mods = {m: importlib.import_module(m) for m in ("attention", "encoder", "dataset", "model")}
        client = importlib.import_module("client") if with_client else None
    finally:
        sys.path.remove(path)
        for m in list(_MODULES) + list(stubs):
            sys.modules.pop(m, None)
        sys.modules.update(saved)
    return Reference(mods["attention"], mods["encoder"], mods["dataset"], mods["model"], client)


def hf_config(backbone, dropout: float = 0.0):
    """A ``DistilBertConfig`` with the widths of our ``BackboneConfig`` (eager attention, so
    the all-masked ``<unk>`` title row softmaxes over ``finfo.min`` exactly as HF does)."""
    from transformers import DistilBertConfig

    return DistilBertConfig(vocab_size=backbone.vocab_size, dim=backbone.dim, n_layers=backbone.n_layers,
                            n_heads=backbone.n_heads, hidden_dim=backbone.hidden_dim,
                            max_position_embeddings=backbone.max_position, dropout=dropout,
                            attention_dropout=dropout, attn_implementation="eager")


@contextlib.contextmanager
def random_init_backbone(backbone, dropout: float = 0.0) -> Iterator[None]:
    """Within the block, ``DistilBertModel.from_pretrained(...)`` returns a random-init model
    of our backbone's shape (no pretrained weights offline)."""
    from transformers import DistilBertModel

    own = DistilBertModel.__dict__.get("from_pretrained")  # usually inherited from PreTrainedModel
    DistilBertModel.from_pretrained = classmethod(lambda cls, *a, **k: cls(hf_config(backbone, dropout)))
    try:
        yield
    finally:
        if own is None:
            del DistilBertModel.from_pretrained
        else:
            DistilBertModel.from_pretrained = own


def user_model(ref: Reference, ours, news_index, dropout: float = 0.0, user_dropout: float = 0.0):
    """The reference ``UserModel`` (``model.py:10-34``) on the CPU holding OUR weights.
    ``ours``: a ``FedRecModel`` (its state_dict keys are the reference's)."""
    import torch

    with random_init_backbone(ours.cfg.backbone, dropout):
        um = ref.model.UserModel(None, news_index, torch.device("cpu"))
    missing, unexpected = um.load_state_dict(ours.state_dict(), strict=False)
    # HF registers no persistent buffers that we lack beyond position ids; every parameter matches
    params = {n for n, _ in um.named_parameters()}
    assert not [k for k in missing if k in params], missing
    assert not unexpected, unexpected
    um.user_encoder.dropout_rate = user_dropout  # encoder.py:43,50 (hard-coded 0.2)
    return um
