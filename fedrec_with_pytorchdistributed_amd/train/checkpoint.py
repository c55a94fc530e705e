"""Checkpoints in the reference layout.

* ``snapshot.pt``: ``{"MODEL_STATE": state_dict, "EPOCHS_RUN": int}`` -- exactly the two keys
  the reference reads (``client.py:133-147``), with the same 116-key fp32 state_dict, so a
  reference snapshot loads here and ours loads there.  Optional extra keys the reference
  ignores: ``NEXT_EPOCH``, ``OPTIM_STATE`` (flat Adam m/v/step), ``ROUND``, ``RNG``,
  ``CONFIG``.
* resume (Q14): the reference restarts *at* ``EPOCHS_RUN`` (re-running the saved epoch);
  here resumption starts at ``NEXT_EPOCH`` (written explicitly), or ``EPOCHS_RUN + 1`` for
  a reference-written file.
* writes are atomic (tmp file + ``os.replace``) and done by one rank only (the reference
  has every DDP rank write the same file concurrently, ``Gradient_Averaging_main.py:140``).
* ``model.pt`` / ``received_model_{k}.pt`` / ``global_model_round{r}.pt``: raw state_dicts.

Loading always uses ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch

from ..models.fedrec_model import FedRecModel


def cpu_state_dict(model: FedRecModel) -> Dict[str, torch.Tensor]:
    return {k: v.detach().to("cpu", torch.float32).clone() for k, v in model.state_dict().items()}


def atomic_save(obj: Any, path: str) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def rng_state() -> Dict[str, Any]:
    """Host and device torch generator states (user dropout, host sampling fallbacks)."""
    st: Dict[str, Any] = {"RNG": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["RNG_CUDA"] = torch.cuda.get_rng_state_all()
    return st


def restore_rng(snap: Dict[str, Any]) -> bool:
    """Restore what :func:`rng_state` saved; device states only onto the same device count."""
    done = False
    if isinstance(snap.get("RNG"), torch.Tensor):
        torch.set_rng_state(snap["RNG"])
        done = True
    cu = snap.get("RNG_CUDA")
    if cu is not None and torch.cuda.is_available() and len(cu) == torch.cuda.device_count():
        torch.cuda.set_rng_state_all(cu)
    return done


def save_snapshot(path: str, model: FedRecModel, epoch: int, *, round_idx: Optional[int] = None,
                  optim: bool = True, config: Optional[dict] = None,
                  engine: Optional[Dict[str, int]] = None, server_opt: Optional[Dict[str, Any]] = None) -> None:
    """``engine``: the engine's own counters (Philox offsets of LDP noise / dropout, sampler
    epoch) so a resumed run draws fresh randomness instead of replaying the saved one.
    ``server_opt``: the server-side step's state (train/federated.py ServerStep), if any."""
    snap: Dict[str, Any] = {"MODEL_STATE": cpu_state_dict(model), "EPOCHS_RUN": int(epoch),
                            "NEXT_EPOCH": int(epoch) + 1}
    if server_opt:
        snap["SERVER_OPT"] = {k: (v.detach().cpu() if isinstance(v, torch.Tensor) else v)
                              for k, v in server_opt.items()}
    if optim and model.flat is not None:
        snap["OPTIM_STATE"] = model.flat.state()
    if round_idx is not None:
        snap["ROUND"] = int(round_idx)
    snap.update(rng_state())
    if engine is not None:
        snap["ENGINE"] = {k: int(v) for k, v in engine.items()}
    if config is not None:
        snap["CONFIG"] = config
    atomic_save(snap, path)


def load_snapshot(path: str, model: FedRecModel, map_location="cpu", rng: bool = True) -> Dict[str, Any]:
    """Load a snapshot (ours or the reference's) into ``model`` -- parameters, Adam moments
    and step, the torch RNG states -- and return the resume info."""
    snap = torch.load(path, map_location=map_location, weights_only=True)
    if "MODEL_STATE" not in snap:
        raise ValueError(f"{path}: not a snapshot (no MODEL_STATE)")
    model.load_state_dict(snap["MODEL_STATE"])
    if "OPTIM_STATE" in snap and model.flat is not None:
        model.flat.load_state(snap["OPTIM_STATE"])
    restored = restore_rng(snap) if rng else False
    nxt = int(snap.get("NEXT_EPOCH", int(snap["EPOCHS_RUN"]) + 1))
    return {"epochs_run": int(snap["EPOCHS_RUN"]), "next_epoch": nxt, "round": snap.get("ROUND"),
            "rng_restored": restored, "engine": snap.get("ENGINE", {}), "server_opt": snap.get("SERVER_OPT")}


def client_snapshot_path(snapshot_path: str, client: int) -> str:
    """Per-client snapshot of a star-mode client (``client{k}_snapshot.pt`` beside the
    coordinator's ``snapshot.pt``): the reference client auto-loads its own ``snapshot.pt``
    at start (``client.py:125-127``); here every client resumes its Adam state from its file."""
    d, f = os.path.split(snapshot_path)
    return os.path.join(d, f"client{client}_{f}")


def save_client_state(path: str, model: FedRecModel, round_idx: int, engine: Dict[str, int]) -> None:
    """A star client's resume state: the trainable flat parameters, Adam moments + step, RNG
    states and engine counters -- NOT the frozen backbone (the round's global model and the
    client's own seed / checkpoint restore that).  ~14 MB instead of a 270 MB state_dict."""
    snap: Dict[str, Any] = {"FLAT_PARAMS": model.flat.flat.detach().cpu(), "OPTIM_STATE": model.flat.state(),
                            "ROUND": int(round_idx), "ENGINE": {k: int(v) for k, v in engine.items()},
                            "FLAT_NAMES": list(model.flat.names)}
    snap.update(rng_state())
    atomic_save(snap, path)


def load_client_state(path: str, model: FedRecModel) -> Dict[str, Any]:
    snap = torch.load(path, map_location="cpu", weights_only=True)
    if "FLAT_PARAMS" not in snap:  # a full snapshot (round-2 format)
        return load_snapshot(path, model)
    if list(snap.get("FLAT_NAMES", model.flat.names)) != list(model.flat.names):
        raise ValueError(f"{path}: trainable parameter set differs from the model's")
    with torch.no_grad():
        model.flat.flat.copy_(snap["FLAT_PARAMS"].to(model.flat.flat.device))
    model.flat.load_state(snap["OPTIM_STATE"])
    restore_rng(snap)
    return {"round": snap.get("ROUND"), "engine": snap.get("ENGINE", {})}


def save_state_dict(path: str, model: FedRecModel) -> None:
    atomic_save(cpu_state_dict(model), path)


def load_state_dict(path: str) -> Dict[str, torch.Tensor]:
    return torch.load(path, map_location="cpu", weights_only=True)


def flat_to_state_dict(model: FedRecModel, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
    """Full state_dict with the trainable tensors taken from ``flat`` (a flat fp32 buffer
    in ``model.flat`` layout) -- e.g. a received global model in reference format."""
    sd = cpu_state_dict(model)
    f = flat.detach().to("cpu", torch.float32)
    for name, p, off in model.flat.views():
        sd[name] = f[off:off + p.numel()].view(p.shape).clone()
    return sd
