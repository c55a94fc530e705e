"""Where the host time of the config-2 training loop goes (cProfile over bench.py's loop: step
launch + next-batch prepare), to find what bounds the loop once the device step gets shorter.

    python benchmarks/host_profile.py --steps 300 [--top 30]

Prints the per-step host time of the loop and the top functions by own time (per step, us)."""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from fedrec_with_pytorchdistributed_amd.config import FedRecConfig
from fedrec_with_pytorchdistributed_amd.data.synthetic import SynthSpec, SyntheticCorpus
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = FedRecConfig(mode="grad_avg", batch_size=64, seed=0)
    torch.manual_seed(0)
    model = FedRecModel(cfg).to(dev)
    model.build_flat()
    shard = SyntheticCorpus(SynthSpec.preset("mind-small")).client_shard(0, 1)
    eng = LocalEngine(cfg, model, shard, dev)
    eng.build_cache()
    it = iter(eng.sampler.epoch(0))

    def nxt():
        nonlocal it
        p = eng._next_prepared(it)
        if p is None:
            it = iter(eng.sampler.epoch(1))
            p = eng._next_prepared(it)
        return p

    pre = nxt()
    for _ in range(a.warmup):
        eng.train_prepared(pre)
        pre = nxt()
    torch.cuda.synchronize()

    def loop(n):
        nonlocal pre
        for _ in range(n):
            eng.train_prepared(pre)
            pre = nxt()

    t0 = time.perf_counter()
    loop(a.steps)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    pr = cProfile.Profile()
    pr.enable()
    loop(a.steps)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    rows = []
    for (fn, line, name), (cc, nc, tt, ct, _) in st.stats.items():
        rows.append((tt / a.steps * 1e6, ct / a.steps * 1e6, nc / a.steps, f"{os.path.basename(fn)}:{line}:{name}"))
    rows.sort(reverse=True)
    print(f"wall per step (unprofiled) {wall * 1e3:.4f} ms; profiled top by own time, us per step "
          f"(own, cumulative, calls):")
    for r in rows[: a.top]:
        print(f"{r[0]:9.1f} {r[1]:9.1f} {r[2]:6.1f}  {r[3]}")


if __name__ == "__main__":
    main()
