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
            _apply_env_knobs(torch.ops.fedrec)
    return torch.ops.fedrec


def _apply_env_knobs(ops) -> None:
    """Kernel-variant switches for A/B runs (unset = the measured defaults)."""
    if os.environ.get("FEDREC_LN_WIDE"):
        ops.ln_set_wide(int(os.environ["FEDREC_LN_WIDE"]))
    if os.environ.get("FEDREC_SCORE_VARIANT"):
        ops.score_set_variant(int(os.environ["FEDREC_SCORE_VARIANT"]))
    if os.environ.get("FEDREC_UA_VARIANT"):
        ops.user_attn_set_variant(int(os.environ["FEDREC_UA_VARIANT"]))
    if os.environ.get("FEDREC_TA_WAVES"):
        ops.title_attn_set_waves(int(os.environ["FEDREC_TA_WAVES"]))
    if os.environ.get("FEDREC_TAB_VARIANT"):
        ops.title_attn_bwd_set_variant(int(os.environ["FEDREC_TAB_VARIANT"]))
    if os.environ.get("FEDREC_TAB_DROP_SPLIT"):
        ops.title_attn_bwd_set_variant(10 + int(os.environ["FEDREC_TAB_DROP_SPLIT"]))
    if os.environ.get("FEDREC_SEGSUM_VARIANT"):
        ops.segsum_set_variant(int(os.environ["FEDREC_SEGSUM_VARIANT"]))
    if os.environ.get("FEDREC_GEMM_VARIANT"):
        ops.gemm_set_variant(int(os.environ["FEDREC_GEMM_VARIANT"]))


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
