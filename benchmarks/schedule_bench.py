"""ms per local step of the two local-update schedules on one GPU (same shard, same batches):
per_step (GA / PA: Adam every step) vs per_epoch (star FedAvg: per-news gradient table,
replay + Adam at epoch end).  Usage: python benchmarks/schedule_bench.py [--steps 200]."""
import argparse
import json
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))

import torch

from fedrec_with_pytorchdistributed_amd.config import FedRecConfig
from fedrec_with_pytorchdistributed_amd.data.synthetic import SynthSpec, SyntheticCorpus
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--preset", default="mind-small")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    shard = SyntheticCorpus(SynthSpec.preset(a.preset)).client_shard(0, 1)
    for sched, mode in (("per_step", "grad_avg"), ("per_epoch", "fedavg_star"), ("per_step", "grad_avg")):
        cfg = FedRecConfig(mode=mode, batch_size=64)
        cfg.local_update = sched
        torch.manual_seed(0)
        m = FedRecModel(cfg).to(dev)
        m.build_flat()
        eng = LocalEngine(cfg, m, shard, dev)
        eng.train_epoch(max_steps=10)  # warm-up (allocator, first-touch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = eng.train_epoch(max_steps=a.steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"schedule": sched, "steps": st["steps"], "ms_per_step_incl_epoch_end": round(1000 * dt / st["steps"], 3)}),
              flush=True)


if __name__ == "__main__":
    main()
