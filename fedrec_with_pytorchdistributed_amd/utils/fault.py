"""Fault injection for failure-detection tests (the reference has none).

``FEDREC_FAULT`` holds comma-separated rules ``<role>:<index>:round:<r>:<action>[:<arg>]``:

* ``kill``  -- the process exits immediately (a client vanishing mid-round);
* ``hang``  -- the process stops making progress (sleeps), like a wedged peer;
* ``nan``   -- the client's upload is poisoned with NaNs;
* ``slow:<s>`` -- sleep ``s`` seconds before uploading (a straggler).

Example: ``FEDREC_FAULT=client:1:round:2:kill,client:0:round:3:nan``.  The coordinator must
answer with a quorum aggregation (or a clean abort) within ``round_timeout_s`` -- never the
reference's 2-day hang.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import List, Optional

import torch


@dataclass
class Rule:
    role: str
    index: int
    round: int
    action: str
    arg: float = 0.0


def parse(spec: str) -> List[Rule]:
    rules = []
    for item in filter(None, (s.strip() for s in spec.split(","))):
        p = item.split(":")
        if len(p) < 5 or p[2] != "round":
            raise ValueError(f"bad FEDREC_FAULT rule {item!r}")
        rules.append(Rule(p[0], int(p[1]), int(p[3]), p[4], float(p[5]) if len(p) > 5 else 0.0))
    return rules


class FaultInjector:
    def __init__(self, role: str, index: int, spec: Optional[str] = None):
        spec = os.environ.get("FEDREC_FAULT", "") if spec is None else spec
        self.rules = [r for r in parse(spec) if r.role == role and r.index == index]

    def _match(self, round_idx: int) -> Optional[Rule]:
        for r in self.rules:
            if r.round == round_idx:
                return r
        return None

    def before_upload(self, round_idx: int, flat: Optional[torch.Tensor] = None) -> None:
        r = self._match(round_idx)
        if r is None:
            return
        if r.action == "kill":
            os._exit(3)
        if r.action == "hang":
            while True:
                time.sleep(3600)
        if r.action == "slow":
            time.sleep(r.arg)
        if r.action == "nan" and flat is not None:
            flat.fill_(float("nan"))
