"""Device time between back-to-back replays of the config-2 STEP graph (no host work, no
lookahead, no eager kernel in between): per-replay wall time from events against the replay's
kernel time.  Under ``rocprofv3 --kernel-trace`` the seam shows as idle between one replay's
last kernel (adam_dev) and the next replay's first.

    python benchmarks/graph_seam.py --replays 40
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from fedrec_with_pytorchdistributed_amd.config import FedRecConfig
from fedrec_with_pytorchdistributed_amd.data.synthetic import SynthSpec, SyntheticCorpus
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replays", type=int, default=40)
    ap.add_argument("--preset", default="mind-small")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = FedRecConfig(mode="grad_avg", batch_size=64, seed=0)
    torch.manual_seed(0)
    model = FedRecModel(cfg).to(dev)
    model.build_flat()
    shard = SyntheticCorpus(SynthSpec.preset(a.preset)).client_shard(0, 1)
    eng = LocalEngine(cfg, model, shard, dev)
    eng.build_cache()
    it = iter(eng.sampler.epoch(0))
    pre = eng._next_prepared(it)
    for _ in range(6):  # capture + warm the step graphs
        eng.train_prepared(pre)
        pre = eng._next_prepared(it)
    torch.cuda.synchronize()
    g = next(v for k, v in eng._graphs.items() if k[-2])  # a graph with Adam inside
    res = {}
    x = torch.zeros(1024, device=dev)
    for name, fn in (("replay", lambda: g.graph.replay()),
                     ("eager_kernel_plus_replay", lambda: (x.add_(1.0), g.graph.replay()))):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.replays):
            fn()
        e.record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(s.elapsed_time(e) * 1000.0 / a.replays, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    sys.exit(main())
