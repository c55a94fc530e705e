"""Loader for the in-tree HIP extension (``_C.so``, built by ``csrc/build.py`` for gfx950).

Ops register under ``torch.ops.fedrec`` via ``TORCH_LIBRARY``.  The extension is loaded
once; on a machine with a GPU a missing or stale extension is a hard error (no silent
eager fallback -- the round-end driver checks which native code the GPU tests load).
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

PKG_DIR = Path(__file__).resolve().parent.parent
SO_PATH = PKG_DIR / "_C.so"

_lock = threading.Lock()
_loaded = False
_error: Exception | None = None


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def lib():
    """Return ``torch.ops.fedrec`` after loading ``_C.so`` (raises if it cannot be loaded)."""
    global _loaded, _error
    if _loaded:
        return torch.ops.fedrec
    with _lock:
        if not _loaded:
            if _error is not None:
                raise _error
            if not SO_PATH.exists():
                _error = RuntimeError(
                    f"HIP extension {SO_PATH} is missing: run `python -m "
                    f"fedrec_with_pytorchdistributed_amd.csrc.build` (or __graft_entry__.build())")
                raise _error
            try:
                torch.ops.load_library(str(SO_PATH))
            except Exception as e:  # pragma: no cover - depends on the box
                _error = RuntimeError(f"failed to load {SO_PATH}: {e}")
                raise _error
            _loaded = True
    return torch.ops.fedrec


def require_for(t: torch.Tensor):
    """The HIP op table for a device tensor; raises loudly when it is unavailable."""
    if not t.is_cuda:
        raise RuntimeError("HIP ops need a device tensor")
    return lib()


def no_kernel(op: str, t: torch.Tensor):
    """A device tensor reached an op that has no HIP kernel for its dtype: fail loudly (the
    engine never silently runs a torch-eager replacement on the device)."""
    raise RuntimeError(f"fedrec::{op}: no HIP kernel for {t.dtype} device tensors (the device path is bf16; "
                       f"--precision=fp32 runs on the host only)")
