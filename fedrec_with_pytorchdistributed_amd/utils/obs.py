"""Observability: roctx ranges, JSONL metrics, per-phase timers, optional wandb.

The reference has only ``print`` and a disabled wandb run with a committed API key
(``client.py:214-219``, C40).  Here:

* :func:`range` emits a roctx range (``libroctx64``, visible in ``rocprofv3
  --marker-trace`` / kernel traces) around each phase when ``FEDREC_ROCTX=1``;
* :class:`MetricsWriter` appends one JSON object per record (rank 0 / coordinator);
  metric names keep the reference's six wandb keys (``training_loss``,
  ``validation_loss``, ``valid_auc``, ``valid_mrr``, ``val_ndcg@5``, ``val_ndcg@10``);
* wandb is used only when ``FEDREC_WANDB=1`` *and* it is importable; no key is ever
  embedded (login comes from the environment).
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import sys
import time
from typing import Any, Dict, Optional

_roctx = None
_roctx_tried = False


def _load_roctx():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if os.environ.get("FEDREC_ROCTX", "0") != "1":
        return None
    for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctxRange naming
    lib = _load_roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


_VERBOSE = os.environ.get("FEDREC_QUIET", "0") != "1"


def log(msg: str) -> None:
    if _VERBOSE:
        print(msg, file=sys.stderr, flush=True)


class MetricsWriter:
    def __init__(self, path: Optional[str], run_name: str = "fedrec", project: str = "Node4",
                 config: Optional[Dict[str, Any]] = None):
        self.path = path
        self._wandb = None
        if path:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
        if os.environ.get("FEDREC_WANDB", "0") == "1":
            try:  # pragma: no cover - wandb is not installed in this image
                import wandb

                wandb.init(project=project, name=run_name, config=config or {})
                self._wandb = wandb
            except Exception as e:  # pragma: no cover
                log(f"wandb unavailable: {e}")

    def write(self, record: Dict[str, Any]) -> None:
        rec = {"ts": time.time(), **record}
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(rec, default=float) + "\n")
        if self._wandb is not None:  # pragma: no cover
            self._wandb.log({k: v for k, v in record.items() if isinstance(v, (int, float))})


class Timer:
    def __init__(self):
        self.t: Dict[str, float] = {}

    @contextlib.contextmanager
    def __call__(self, name: str, sync=None):
        if sync is not None:
            sync()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if sync is not None:
                sync()
            self.t[name] = self.t.get(name, 0.0) + time.perf_counter() - t0
