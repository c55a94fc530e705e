"""Control plane on the c10d key-value store (the torchrun rendezvous store).

The reference coordinates rounds with gloo collectives (a 0-d flag broadcast from a
hard-coded ``src=1``, ``client.py:256-264``) and moves models over a raw TCP socket with
no framing, retries or timeouts (``client.py:191-210``, ``server.py:25-35``); one dead
client blocks the server forever (``server.py:89``, Final_Report p.4 §VII.2.a).

Here every round message is a key in the store:

* no collective involves a client after start-up, so a client that dies or hangs costs the
  coordinator one ``round_timeout`` and a quorum decision instead of a deadlock;
* tensors travel as framed blobs (header: dtype, shape, sha256) -- a corrupted or
  truncated upload is detected and dropped;
* keys are prefixed with a run id and round index, so a restarted run never reads stale
  state from an earlier incarnation.
"""
from __future__ import annotations

import hashlib
import io
import json
import struct
import time
from datetime import timedelta
from typing import Dict, Iterable, List, Optional

import numpy as np
import torch
import torch.distributed as dist

_DTYPES = {torch.float32: "f4", torch.int32: "i4", torch.int64: "i8", torch.bfloat16: "bf16", torch.float16: "f2",
           torch.uint8: "u1"}
_RDTYPES = {v: k for k, v in _DTYPES.items()}


def encode_tensor(t: torch.Tensor) -> bytes:
    t = t.detach().contiguous().cpu()
    raw = t.view(torch.uint8).numpy().tobytes() if t.numel() else b""
    hdr = json.dumps({"dtype": _DTYPES[t.dtype], "shape": list(t.shape),
                      "sha256": hashlib.sha256(raw).hexdigest()}).encode()
    return struct.pack("<I", len(hdr)) + hdr + raw


class CorruptBlob(ValueError):
    pass


def decode_tensor(b: bytes) -> torch.Tensor:
    if len(b) < 4:
        raise CorruptBlob("short blob")
    (n,) = struct.unpack("<I", b[:4])
    hdr = json.loads(b[4:4 + n].decode())
    raw = b[4 + n:]
    if hashlib.sha256(raw).hexdigest() != hdr["sha256"]:
        raise CorruptBlob("checksum mismatch")
    dt = _RDTYPES[hdr["dtype"]]
    if len(raw) == 0:
        return torch.empty(hdr["shape"], dtype=dt)
    u8 = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy())
    return u8.view(dt).reshape(hdr["shape"])


class ControlPlane:
    def __init__(self, store: Optional[dist.Store] = None, run_id: str = "fedrec", timeout_s: float = 600.0):
        if store is None:
            store = dist.HashStore()
        self.store = dist.PrefixStore(f"fedrec/{run_id}/", store)
        self.timeout_s = timeout_s

    @staticmethod
    def from_default(run_id: str, timeout_s: float) -> "ControlPlane":
        st = None
        if dist.is_available() and dist.is_initialized():
            st = dist.distributed_c10d._get_default_store()
        return ControlPlane(st, run_id, timeout_s)

    # --- bytes ------------------------------------------------------------------------
    def set(self, key: str, value: bytes | str) -> None:
        self.store.set(key, value if isinstance(value, bytes) else value.encode())

    def has(self, key: str) -> bool:
        return self.store.check([key])

    def get(self, key: str, timeout_s: Optional[float] = None) -> bytes:
        """Block until ``key`` exists (or raise TimeoutError)."""
        t = self.timeout_s if timeout_s is None else timeout_s
        deadline = time.monotonic() + t
        while not self.store.check([key]):
            if time.monotonic() > deadline:
                raise TimeoutError(f"control plane: {key!r} not set within {t:.0f}s")
            time.sleep(0.02)
        return self.store.get(key)

    def wait_any(self, keys: Iterable[str], need: int, timeout_s: float, poll_s: float = 0.05) -> List[str]:
        """Wait until all keys exist, or until the timeout with at least ``need`` present.
        Returns the present keys (may be fewer than ``need`` on timeout)."""
        keys = list(keys)
        deadline = time.monotonic() + timeout_s
        while True:
            present = [k for k in keys if self.store.check([k])]
            if len(present) == len(keys) or time.monotonic() > deadline:
                return present
            time.sleep(poll_s)

    def add(self, key: str, n: int = 1) -> int:
        return int(self.store.add(key, n))

    # --- tensors / json ---------------------------------------------------------------
    def put_tensor(self, key: str, t: torch.Tensor) -> None:
        self.set(key, encode_tensor(t))

    def get_tensor(self, key: str, timeout_s: Optional[float] = None) -> torch.Tensor:
        return decode_tensor(self.get(key, timeout_s))

    def put_json(self, key: str, obj: Dict) -> None:
        self.set(key, json.dumps(obj, default=float))

    def get_json(self, key: str, timeout_s: Optional[float] = None) -> Dict:
        return json.loads(self.get(key, timeout_s).decode())

    # --- heartbeats ----------------------------------------------------------------------
    # A heartbeat is a progress COUNTER, not a timestamp: the coordinator times how long a
    # counter has stood still on its own monotonic clock, so client clock skew across nodes
    # cannot fake liveness or death.
    def heartbeat(self, who: str) -> int:
        return self.add(f"hb/{who}", 1)

    def heartbeat_count(self, who: str) -> int:
        k = f"hb/{who}"
        return int(self.store.get(k).decode()) if self.store.check([k]) else 0

    def wait_uploads(self, keys: Dict[int, str], need: int, timeout_s: float, hb_timeout_s: float = 0.0,
                     who=lambda k: f"client{k}", poll_s: float = 0.05, log=None):
        """Wait for every client's upload key, or until each missing client is declared dead
        (heartbeat counter unchanged for ``hb_timeout_s``) with ``need`` uploads present, or
        until ``timeout_s``.  Returns ``(present_keys, dead_clients)``."""
        now = time.monotonic()
        deadline = now + timeout_s
        seen = {k: (self.heartbeat_count(who(k)), now) for k in keys}
        dead: set = set()
        while True:
            present = [k for k in keys if self.store.check([keys[k]])]
            now = time.monotonic()
            if len(present) == len(keys) or now > deadline:
                break
            if hb_timeout_s > 0:
                for k in keys:
                    if k in present or k in dead:
                        continue
                    c = self.heartbeat_count(who(k))
                    if c != seen[k][0]:
                        seen[k] = (c, now)
                    elif now - seen[k][1] > hb_timeout_s:
                        dead.add(k)
                        if log is not None:
                            log(f"client {k}: no heartbeat for {hb_timeout_s:.0f}s (counter {c}); declared dead")
                if dead and all(k in present or k in dead for k in keys):
                    break
            time.sleep(poll_s)
        return [keys[k] for k in keys if k in present], sorted(dead)


class Heartbeat:
    """Client side: ``beat()`` bumps the counter, at most once per ``interval_s``."""

    def __init__(self, cp: ControlPlane, who: str, interval_s: float):
        self.cp, self.who, self.interval = cp, who, interval_s
        self._last = -1e30

    def __call__(self, *_args, force: bool = False) -> None:
        if self.interval <= 0 and not force:
            return
        now = time.monotonic()
        if force or now - self._last >= self.interval:
            self._last = now
            self.cp.heartbeat(self.who)
