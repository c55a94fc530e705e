"""All-reduce sweep over the data-plane process group (RCCL over xGMI on a GPU node, gloo on
CPU): message sizes from 4 KB to 256 MB, time per call and bus bandwidth
(2 (W-1)/W x bytes / time, the rccl-tests convention).  The engine's buckets are marked:
the GA step's flat trainable gradient (4.66 MB fp32) and the ``sync=full`` 28 MB buckets.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/allreduce_bench.py [--max-mb 256]

Rank 0 prints one JSON line per size.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.distributed as dist

from fedrec_with_pytorchdistributed_amd.parallel import dist as fdist

MARKS = {1_164_882 * 4: "GA flat gradient bucket", 28 << 20: "sync=full bucket"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-kb", type=float, default=4)
    ap.add_argument("--max-mb", type=float, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16", "int32"])
    a = ap.parse_args()
    ctx = fdist.init("client", "auto", timeout_s=600)
    W = ctx.world
    dt = getattr(torch, a.dtype)
    esz = torch.empty(0, dtype=dt).element_size()
    sizes = []
    b = int(a.min_kb * 1024)
    while b <= a.max_mb * (1 << 20):
        sizes.append(b)
        b *= 4
    sizes = sorted(set(sizes) | {s for s in MARKS if s <= a.max_mb * (1 << 20)})
    dev = ctx.device
    group = ctx.data_group

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for nbytes in sizes:
        n = max(1, nbytes // esz)
        t = torch.ones(n, dtype=dt, device=dev)
        for _ in range(a.warmup):
            if ctx.initialized:
                dist.all_reduce(t, group=group)
        sync()
        if ctx.initialized:
            dist.barrier(group=ctx.ctrl_group)
        t0 = time.perf_counter()
        for _ in range(a.iters):
            if ctx.initialized:
                dist.all_reduce(t, group=group)
        sync()
        el = (time.perf_counter() - t0) / a.iters
        if ctx.initialized:
            m = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=ctx.ctrl_group)
            el = float(m.item())
        if ctx.rank == 0:
            busbw = 2.0 * (W - 1) / max(W, 1) * n * esz / el / 1e9 if W > 1 else 0.0
            print(json.dumps({"bytes": n * esz, "world": W, "dtype": a.dtype, "us": round(el * 1e6, 2),
                              "busbw_GBps": round(busbw, 2), "backend": "rccl" if dev.type == "cuda" else "gloo",
                              "note": MARKS.get(nbytes, "")}), flush=True)
    fdist.shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
