"""AUC A/B: the reference's own training loop vs this engine, same shard, same weights.

Both sides start from the same random-init weights (ours, loaded into the reference
``UserModel`` by :mod:`fedrec_with_pytorchdistributed_amd.eval.refharness`), see the same
batches (our host sampler; the reference's ``TrainDataset`` draws unseeded negatives,
``dataset.py:14``) and run star-client local epochs on the CPU in fp32:

* reference: ``client.train_on_step`` (``client.py:61-101``) -> ``UserModel.update``, then the
  validation forward of ``Trainer.validate`` (``client.py:149-171``: B = 1, candidates
  ``[pos] + negs[-4:]``) scored with the reference's ``evaluation_functions`` -- reported as
  the corpus mean over impressions (its Q9 "last impression only" value alongside);
* ours: ``LocalEngine.train_epoch`` (per-epoch schedule, ``compat.reference_quirks=1``) and
  ``LocalEngine.validate`` on the same validation impressions.

Dropout is off on both sides by default (``--dropout`` turns the reference's user dropout
0.2 / DistilBERT 0.1 and ours on; the masks then differ, so the runs are statistically, not
numerically, comparable).

    python benchmarks/ref_auc_ab.py --preset tiny --backbone tiny --epochs 3 --lr 5e-5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fedrec_with_pytorchdistributed_amd.config import BackboneConfig, FedRecConfig  # noqa: E402
from fedrec_with_pytorchdistributed_amd.data.sampler import HostSampler, validation_batches  # noqa: E402
from fedrec_with_pytorchdistributed_amd.data.synthetic import make_client_shards  # noqa: E402
from fedrec_with_pytorchdistributed_amd.eval import refharness  # noqa: E402
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel  # noqa: E402
from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine  # noqa: E402


def ref_validate(ref, um, shard, limit):
    """``Trainer.validate`` (client.py:149-171) without its Trainer: one forward per impression,
    metrics from the reference's evaluation_functions, corpus mean + the last impression."""
    ev = ref.client  # client.py imports roc_auc_score, mrr_score, ndcg_score from evaluation_functions
    um.eval()
    aucs, mrrs, n5, n10, losses = [], [], [], [], []
    for cand, his in validation_batches(shard.valid, 1, 4, 50, True, limit):
        c = torch.from_numpy(cand).long()
        h = torch.from_numpy(his).long()
        with torch.no_grad():
            loss, score, _, _ = um(c, h, torch.zeros(1, dtype=torch.long))
        y = np.array([1, 0, 0, 0, 0])
        s = score.reshape(-1).numpy()
        aucs.append(ev.roc_auc_score(y, s))
        mrrs.append(ev.mrr_score(y, s))
        n5.append(ev.ndcg_score(y, s, k=5))
        n10.append(ev.ndcg_score(y, s, k=10))
        losses.append(float(loss))
    return {"valid_auc": float(np.mean(aucs)), "valid_mrr": float(np.mean(mrrs)),
            "val_ndcg@5": float(np.mean(n5)), "val_ndcg@10": float(np.mean(n10)),
            "validation_loss": float(np.mean(losses)), "last_valid_auc": float(aucs[-1]), "n_valid": len(aucs)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="tiny")
    ap.add_argument("--backbone", default="tiny")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--lr", type=float, default=5e-5)
    ap.add_argument("--max-steps", type=int, default=0, help="cap batches per epoch (0 = whole shard)")
    ap.add_argument("--valid-limit", type=int, default=200)
    ap.add_argument("--score-act", default="sigmoid")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    torch.set_num_threads(8)

    ref = refharness.load()
    shard = make_client_shards(args.preset, 1)[0]
    cfg = FedRecConfig(mode="fedavg_star", batch_size=args.batch, user_dropout=0.0, lr=args.lr,
                       score_act=args.score_act)
    # the reference's training quirks: Q2 (user grads x2, last batch only), Q4 (train-mode replay);
    # histories are truncated to the last 50 on both sides (synthetic ones reach 90) and both
    # report corpus means (the reference's Q9 last-impression value is printed alongside)
    cfg.compat.grad_double_last_batch = True
    cfg.compat.replay_train_mode = True
    cfg.backbone = BackboneConfig.preset(args.backbone)
    torch.manual_seed(args.seed)
    ours = FedRecModel(cfg)
    ours.build_flat()
    um = refharness.user_model(ref, ours, shard.news_index)
    for opt in (um.user_optimizer, um.news_optimizer):
        for g in opt.param_groups:
            g["lr"] = args.lr  # model.py:22-23 hard-codes 5e-5
    if args.score_act != "sigmoid":
        raise SystemExit("the reference scorer is sigmoid (model.py:123); identity has no reference counterpart")
    eng = LocalEngine(cfg, ours, shard, torch.device("cpu"))
    sampler = HostSampler(shard.train, args.batch, 4, 50, truncate=True, seed=args.seed)
    sgd = torch.optim.SGD(um.parameters(), lr=5e-5)
    rows = []
    r0 = ref_validate(ref, um, shard, args.valid_limit)
    o0 = eng.validate(limit=args.valid_limit)
    rows.append({"epoch": 0, "ref": r0, "ours": {k: o0[k] for k in r0 if k in o0}})
    print(json.dumps(rows[-1]), flush=True)
    for ep in range(args.epochs):
        batches = []
        for i, (c, h) in enumerate(sampler.epoch(ep)):
            if args.max_steps and i >= args.max_steps:
                break
            batches.append((torch.from_numpy(c).long(), torch.from_numpy(h).long()))
        t0 = time.perf_counter()
        um.train()
        r_loss = ref.client.train_on_step(um, [(c, h, torch.zeros(c.shape[0], dtype=torch.long)) for c, h in batches],
                                          sgd, False, 0.0)
        t1 = time.perf_counter()
        eng._begin_epoch_accumulate()
        o_loss = sum(float(eng.accumulate_step(c, h)) for c, h in batches)
        eng.end_epoch_update(len(batches))
        t2 = time.perf_counter()
        rv = ref_validate(ref, um, shard, args.valid_limit)
        ov = eng.validate(limit=args.valid_limit)
        rows.append({"epoch": ep + 1, "steps": len(batches), "ref_train_loss_sum": float(r_loss),
                     "ours_train_loss_sum": o_loss, "ref_epoch_s": round(t1 - t0, 2), "ours_epoch_s": round(t2 - t1, 2),
                     "ref": rv, "ours": {k: ov[k] for k in rv if k in ov}})
        print(json.dumps(rows[-1]), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            for r in rows:
                f.write(json.dumps({**r, "args": vars(args)}) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
