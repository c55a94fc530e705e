"""Run the 2-client shared-GPU rehearsal of the N > 1 step (tests/_graph_ar_worker.py: in-graph
IPC all-reduce, early user-slice reduce) -- meant to run under rocprofv3 --kernel-trace, which
traces both client processes (they inherit its environment)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from launch_util import run_ranks  # noqa: E402

SHARE = {"FEDREC_CPU_ONLY": "0", "FEDREC_SHARE_GPU": "1", "FEDREC_DATA_BACKEND": "gloo", "FEDREC_QUIET": "1"}
W = int(sys.argv[1]) if len(sys.argv) > 1 else 2
outs = run_ranks([["tests/_graph_ar_worker.py"]] * W, SHARE, timeout=400)
for rc, out in outs:
    print(rc, out[-600:])
sys.exit(0 if all(rc == 0 for rc, _ in outs) else 1)
