"""Two-rank worker for test_collective_checker_*: both ranks issue real gloo all-reduces
through parallel.comm; with ``--diverge`` rank 1 reduces one bucket with MAX instead of SUM
(same size, so the transport cannot notice: the silent kind of divergence)."""
import sys

import torch
import torch.distributed as dist

from fedrec_with_pytorchdistributed_amd.parallel import comm
from fedrec_with_pytorchdistributed_amd.parallel.collcheck import CHECK, CollectiveMismatch

dist.init_process_group("gloo")
rank = dist.get_rank()
diverge = "--diverge" in sys.argv
for i in range(5):
    op = dist.ReduceOp.MAX if diverge and rank == 1 and i == 3 else dist.ReduceOp.SUM
    comm.allreduce_([torch.ones(8)], None, op=op)
try:
    CHECK.verify(None, "worker")
    print("COLLCHECK OK", CHECK.count, flush=True)
except CollectiveMismatch as e:
    print("COLLCHECK MISMATCH", str(e).replace("\n", " || "), flush=True)
dist.destroy_process_group()
