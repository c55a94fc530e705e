"""Command-line front end.  The reference's positional contracts are kept verbatim:

* ``client.py <total_epochs> <batch_size> <save_every> <dp_epsilon:int> <run_name>``  (client.py:300-305)
* ``server.py <global_epochs>``                                                  (server.py:113)
* ``Gradient_Averaging_main.py / Parameter_Averaging_main.py / main.py
  <total_epochs> <batch_size> <save_every>``                                      (…_main.py:190-195)

and any trailing ``--key=value`` overrides a :class:`FedRecConfig` field (``--data_dir=...``,
``--dp.epsilon=10``, ``--backbone.name=bert-base``, ``--compat.reference_quirks=1`` ...).

All of them run under ``torchrun`` (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the env), as in
the README recipe (``README.md:24-46``): two torchrun invocations (server node and client
node) join one c10d rendezvous; roles come from the entrypoint, never from rank numbers.
For a one-invocation single-node star run, ``python -m fedrec_with_pytorchdistributed_amd.cli
star <rounds> <epochs> <batch> [--k=v]`` under ``torchrun --nproc-per-node W+1`` makes rank 0
the coordinator and ranks 1..W the GPU clients.
"""
from __future__ import annotations

import os
import sys
from typing import List, Optional

from .config import FedRecConfig


def _cfg(rest: List[str]) -> FedRecConfig:
    cfg = FedRecConfig()
    leftover = cfg.apply_overrides(rest)
    if leftover:
        raise SystemExit(f"unexpected arguments: {leftover}")
    return cfg


def _client_dev_offset() -> int:
    return int(os.environ.get("FEDREC_GPU_OFFSET", "0"))


def main_client(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    pos = [a for a in argv if not a.startswith("--")]
    if len(pos) < 5:
        raise SystemExit("usage: client.py <total_epochs> <batch_size> <save_every> <dp_epsilon> <run_name> [--k=v]")
    cfg = _cfg([a for a in argv if a.startswith("--")])
    cfg.total_epochs, cfg.batch_size, cfg.save_every = int(pos[0]), int(pos[1]), int(pos[2])
    eps = int(pos[3])
    cfg.dp.epsilon, cfg.dp.enabled = float(eps), bool(eps)  # dp_enabled = bool(dp_Epsilon) (client.py:304)
    cfg.run_name = pos[4]
    cfg.mode = "fedavg_star"
    from .parallel import dist as fdist
    from .train.federated import run_star_client

    ctx = fdist.init("client", cfg.device, cfg.collective_timeout_s, gpu_offset=_client_dev_offset())
    try:
        run_star_client(cfg, ctx)
    finally:
        fdist.shutdown(ctx)
    return 0


def main_server(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    pos = [a for a in argv if not a.startswith("--")]
    if len(pos) < 1:
        raise SystemExit("usage: server.py <global_epochs> [--k=v]")
    cfg = _cfg([a for a in argv if a.startswith("--")])
    cfg.global_rounds = int(pos[0])
    cfg.mode = "fedavg_star"
    from .parallel import dist as fdist
    from .train.federated import run_star_server

    ctx = fdist.init("server", "cpu", cfg.collective_timeout_s)
    try:
        run_star_server(cfg, ctx)
    finally:
        fdist.shutdown(ctx)
    return 0


def _main_dp(mode: str, argv: Optional[List[str]]) -> int:
    argv = sys.argv[1:] if argv is None else argv
    pos = [a for a in argv if not a.startswith("--")]
    if len(pos) < 3:
        raise SystemExit("usage: <total_epochs> <batch_size> <save_every> [--k=v]")
    cfg = _cfg([a for a in argv if a.startswith("--")])
    cfg.total_epochs, cfg.batch_size, cfg.save_every = int(pos[0]), int(pos[1]), int(pos[2])
    cfg.mode = mode
    from .parallel import dist as fdist
    from .train.federated import run_grad_avg, run_param_avg

    ctx = fdist.init("client", cfg.device, cfg.collective_timeout_s)
    try:
        (run_grad_avg if mode == "grad_avg" else run_param_avg)(cfg, ctx)
    finally:
        fdist.shutdown(ctx)
    return 0


def main_grad_avg(argv=None) -> int:
    return _main_dp("grad_avg", argv)


def main_param_avg(argv=None) -> int:
    return _main_dp("param_avg", argv)


def main_star(argv: Optional[List[str]] = None) -> int:
    """One torchrun: rank 0 coordinator, ranks 1..W GPU clients."""
    argv = sys.argv[1:] if argv is None else argv
    pos = [a for a in argv if not a.startswith("--")]
    if len(pos) < 3:
        raise SystemExit("usage: star <global_rounds> <local_epochs> <batch_size> [--k=v]")
    rank = int(os.environ.get("RANK", "0"))
    extra = [a for a in argv if a.startswith("--")]
    if rank == 0:
        return main_server([pos[0], *extra])
    os.environ["FEDREC_GPU_OFFSET"] = "1"
    return main_client([pos[1], pos[2], "1", "0", "star", *extra])


COMMANDS = {"client": main_client, "server": main_server, "grad_avg": main_grad_avg, "param_avg": main_param_avg,
            "star": main_star}


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] not in COMMANDS:
        raise SystemExit(f"usage: python -m fedrec_with_pytorchdistributed_amd.cli {{{','.join(COMMANDS)}}} ...")
    return COMMANDS[argv[0]](argv[1:])


if __name__ == "__main__":
    sys.exit(main())
