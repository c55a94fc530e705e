"""Host vs device timeline of the config-2 training loop (bench.py's loop, no profiler):
per step, the host times at which the step's launch starts / returns and the next batch is
prepared, against the device time at which the step's first and last work ran (timing events
recorded on the main stream around each step, aligned to the host clock at a synchronised
start).  A step whose device start follows its host launch closely is host-bound.

    python benchmarks/host_timeline.py --steps 30
"""
import argparse
import json
import os
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
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = FedRecConfig(mode="grad_avg", batch_size=a.batch, seed=0)
    torch.manual_seed(0)
    model = FedRecModel(cfg).to(dev)
    model.build_flat()
    shard = SyntheticCorpus(SynthSpec.preset("mind-small")).client_shard(0, 1)
    eng = LocalEngine(cfg, model, shard, dev)
    eng.build_cache()
    it = iter(eng.sampler.epoch(0))
    pre = eng._next_prepared(it)
    for _ in range(a.warmup):
        eng.train_prepared(pre)
        pre = eng._next_prepared(it)
    torch.cuda.synchronize()
    main_s = torch.cuda.current_stream(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record(main_s)
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    rec = []
    for _ in range(a.steps):
        eb, ee = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t_a = time.perf_counter()
        eb.record(main_s)
        eng.train_prepared(pre)
        ee.record(main_s)
        t_b = time.perf_counter()
        pre = eng._next_prepared(it)
        t_c = time.perf_counter()
        rec.append((t_a, t_b, t_c, eb, ee))
    torch.cuda.synchronize()
    rows = []
    for t_a, t_b, t_c, eb, ee in rec:
        rows.append({"host_launch_us": round((t_a - h0) * 1e6, 1), "host_launched_us": round((t_b - h0) * 1e6, 1),
                     "host_next_batch_us": round((t_c - h0) * 1e6, 1),
                     "dev_start_us": round(e0.elapsed_time(eb) * 1e3, 1), "dev_end_us": round(e0.elapsed_time(ee) * 1e3, 1)})
    for r in rows:
        print(r)
    per = (rows[-1]["dev_end_us"] - rows[0]["dev_start_us"]) / (len(rows) - 1)
    slack = [r["dev_start_us"] - r["host_launched_us"] for r in rows]
    print(f"device period {per:.1f} us; device start - host launch returned (mean) {sum(slack) / len(slack):.1f} us; "
          f"host launch {sum(r['host_launched_us'] - r['host_launch_us'] for r in rows) / len(rows):.1f} us, "
          f"next_batch {sum(r['host_next_batch_us'] - r['host_launched_us'] for r in rows) / len(rows):.1f} us")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
