"""Worker of test_cooperative_cache_*: W clients build the hidden-state cache cooperatively
(1/W of the catalog each + all-gather) and compare it with a local build of their own table.

argv: [--device cpu|cuda] [--preset tiny] [--full-table 0|1] [--perturb none|backbone|tokens]
Prints ``CATALOG OK <max abs diff> <titles encoded> <local titles>`` on success.  ``--perturb``:
the last client changes one backbone weight / one shared title's token row first; every client
must then refuse the cooperative plan (``CATALOG REFUSED <reason>``)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--preset", default="tiny")
    ap.add_argument("--backbone", default="tiny")
    ap.add_argument("--piece", type=int, default=97)
    ap.add_argument("--tol", type=float, default=0.0)
    ap.add_argument("--perturb", default="none")
    a = ap.parse_args()
    import numpy as np
    import torch

    from fedrec_with_pytorchdistributed_amd.config import BackboneConfig, FedRecConfig
    from fedrec_with_pytorchdistributed_amd.data.synthetic import SynthSpec, SyntheticCorpus
    from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
    from fedrec_with_pytorchdistributed_amd.parallel import catalog
    from fedrec_with_pytorchdistributed_amd.parallel import dist as fdist
    from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine

    ctx = fdist.init("client", a.device, timeout_s=120)
    cfg = FedRecConfig(mode="grad_avg", batch_size=8, seed=0)
    cfg.news_cache = "hidden"
    cfg.backbone = BackboneConfig.preset(a.backbone)
    torch.manual_seed(0)
    model = FedRecModel(cfg).to(ctx.device)
    model.build_flat()
    shard = SyntheticCorpus(SynthSpec.preset(a.preset)).client_shard(ctx.client_index, ctx.num_clients)
    eng = LocalEngine(cfg, model, shard, ctx.device, rank=ctx.rank)
    assert eng.hcache is not None
    if a.perturb != "none" and ctx.client_index == ctx.num_clients - 1:
        with torch.no_grad():
            if a.perturb == "backbone":
                w = next(eng.model.text_encoder.DistillBert.parameters())
                w.view(-1)[7] += 1e-3
            else:  # a title every client holds (the union's most shared one): token 1 of its row
                gid = catalog.shard_global_ids(shard)
                row = int(np.nonzero(gid >= 0)[0][0])
                eng.tokens[row, 0, 1] += 1
    plan = catalog.attach(eng, ctx, piece_titles=a.piece)
    if a.perturb != "none":
        assert plan is None and eng.catalog is None and eng.catalog_refused, (plan, eng.catalog_refused)
        print(f"CATALOG REFUSED {eng.catalog_refused}", flush=True)
        fdist.shutdown(ctx)
        return 0
    assert plan is not None and plan.pieces >= 2, plan
    # every title of the union is encoded exactly once, by a client holding it
    tot = torch.tensor([plan.mine.size], dtype=torch.int64)
    import torch.distributed as dist

    dist.all_reduce(tot, group=ctx.ctrl_group)
    assert int(tot.item()) == plan.union, (int(tot.item()), plan.union)
    assert sum(plan.counts) == plan.union
    eng.build_cache()
    coop = eng.hcache.table.clone()
    info = dict(eng.hcache.build_info)
    eng.set_catalog(None, None)
    eng.build_cache()
    local = eng.hcache.table
    assert coop.shape == local.shape, (coop.shape, local.shape)
    diff = float((coop.float() - local.float()).abs().max())
    if a.tol == 0.0:
        assert torch.equal(coop, local), diff
    else:
        assert diff <= a.tol, diff
    print(f"CATALOG OK {diff} {info['titles_encoded']} {shard.num_news} {info}", flush=True)
    fdist.shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
