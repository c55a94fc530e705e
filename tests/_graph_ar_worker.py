"""Worker of test_graph_allreduce_*: W GA clients share one GPU; the flat gradient is summed by
the device-epoch IPC all-reduce INSIDE the step graph (one replay per step: backward,
all-reduce, Adam).  The same steps are then re-run with the all-reduce + Adam eager (outside
the graph, the round-4 path) from the same start, and the two trajectories are compared.  The
hidden-state cache is built cooperatively (1/W of the catalog each, gathered over the data
plane).

Prints ``GRAPH_AR OK <|graph - eager| / |eager|>`` on success."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--preset", default="small")
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    from fedrec_with_pytorchdistributed_amd.config import FedRecConfig
    from fedrec_with_pytorchdistributed_amd.data.synthetic import SynthSpec, SyntheticCorpus
    from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
    from fedrec_with_pytorchdistributed_amd.parallel import catalog
    from fedrec_with_pytorchdistributed_amd.parallel import dist as fdist
    from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine

    ctx = fdist.init("client", "cuda", timeout_s=300)
    dev = ctx.device
    shard = SyntheticCorpus(SynthSpec.preset(a.preset)).client_shard(ctx.client_index, ctx.num_clients)
    cfg = FedRecConfig(mode="grad_avg", batch_size=a.batch, seed=0)
    ar = fdist.make_grad_allreduce(ctx, 120.0, choice="ipc", nelem=1 << 20)
    assert ar.kind == "ipc" and ar.capturable

    def run(graph_ar: bool):
        torch.manual_seed(0)
        model = FedRecModel(cfg).to(dev)
        model.build_flat()
        ar.capturable = graph_ar
        eng = LocalEngine(cfg, model, shard, dev, rank=ctx.rank, grad_allreduce=ar)
        plan = catalog.attach(eng, ctx, piece_titles=1500)
        assert plan is not None and eng.hcache is not None
        eng.build_cache()
        st = eng.train_epoch(max_steps=a.steps)
        eng.sync_params()
        torch.cuda.synchronize(dev)
        return eng, model.flat.flat.detach().clone(), st

    eg, pg, sg = run(True)
    c = eg.counts
    assert c["replays"] == a.steps and c["replays_with_optimizer"] == a.steps, c
    assert c["eager_optimizer_steps"] == 0 and c["eager_steps"] == 0, c
    # the user encoder's slice is reduced early, inside the backward, in every replay (the eager
    # run below issues the same two calls per step: user slice, then head slice)
    assert ar.split and c["early_reduces"] == a.steps, (ar.split, c)
    # the text head's and fc's weight gradients were written into the flat buffer by their
    # backward launches (no end-of-backward copy); the copy path gives the same bits
    from fedrec_with_pytorchdistributed_amd.train import engine as E
    assert eg.inplace_grads >= 2, eg.inplace_grads
    E.INPLACE_HEAD_GRADS = False
    try:
        ec, pc, _ = run(True)
    finally:
        E.INPLACE_HEAD_GRADS = True
    assert ec.inplace_grads == 0 and torch.equal(pc, pg), "in-place head gradients changed the trajectory"
    ee, pe, se = run(False)
    assert ee.counts["replays_with_optimizer"] == 0 and ee.counts["eager_optimizer_steps"] == a.steps, ee.counts
    # every client holds the bitwise-same parameters (graph mode), checked over the control group
    host = pg.cpu()
    outs = [torch.empty_like(host) for _ in range(ctx.num_clients)]
    dist.all_gather(outs, host, group=ctx.ctrl_group)
    for o in outs:
        assert torch.equal(o, host), "clients diverged under the in-graph all-reduce"
    # the two paths run different Adam kernels (device step count vs host) over the same sums:
    # last-bit differences that Adam's normalisation carries further on near-zero coordinates,
    # so the trajectories are compared in norm, as test_graph_step_matches_eager does
    d = float((pg - pe).norm() / pe.norm())
    assert torch.isfinite(pg).all() and d <= 5e-5, (d, float((pg - pe).abs().max()))
    assert abs(sg["training_loss"] - se["training_loss"]) < 1e-4, (sg["training_loss"], se["training_loss"])
    ar.ipc.check()
    print(f"GRAPH_AR OK {d} {c}", flush=True)
    fdist.shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
