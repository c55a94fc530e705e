"""Start N cooperating processes the way torchrun would (RANK/WORLD_SIZE/MASTER_* env), but
as independent OS processes: a rank that exits does not tear the others down, which is what
the fault-injection tests need (a client vanishing mid-round)."""
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(argvs, env_extra=None, timeout=240, cwd=None):
    """argvs[i] = argv (list) of rank i.  Returns [(returncode, output)] per rank; processes
    still running at the timeout are killed (returncode None)."""
    port = free_port()
    procs = []
    # run in a scratch directory so default output paths (metrics.jsonl, snapshots) never
    # land in the source tree; entry scripts are resolved against the repo root
    cwd = cwd or tempfile.mkdtemp(prefix="fedrec_ranks_")
    argvs = [[os.path.join(ROOT, a[0]) if a and a[0].endswith(".py") and not os.path.isabs(a[0]) else a[0], *a[1:]]
             for a in argvs]
    for r, argv in enumerate(argvs):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(len(argvs)), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "FEDREC_CPU_ONLY": "1", "OMP_NUM_THREADS": "1",
                    "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", ""), "FEDREC_QUIET": "0"})
        env.update(env_extra or {})
        procs.append(subprocess.Popen([sys.executable, *argv], cwd=cwd, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    deadline = time.monotonic() + timeout
    outs = []
    for p in procs:
        left = max(1.0, deadline - time.monotonic())
        try:
            out, _ = p.communicate(timeout=left)
            outs.append((p.returncode, out))
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
            outs.append((None, out))
    return outs
