"""Training-quality run with collapse diagnostics (one client, gradient averaging, B = 64).

Per epoch: training loss, validation AUC / MRR, and the quantities that tell a collapse of
the scores apart from slow learning --
* news table: mean |v| over titles and the mean distance to the mean vector ("spread"),
* user vectors (validation): mean |u|,
* scores: mean |s|, and the share of impressions whose 5 scores are all equal (ties = a
  constant scorer: AUC exactly 0.5),
* text-head FC weight / bias norms,
* the eps-softmax cliff (``attention.py:20-22,40-42``: ``exp(s) / (sum exp(s) + 1e-8)``): per
  user-MHSA query row and per user pooling, the max logit; below ln(1e-8) = -18.4 the 1e-8
  term dominates and every weight shrinks as exp(max); below ~-87 they are exactly 0 in fp32
  and so is the gradient through them (an absorbing state).

    python benchmarks/quality_diag.py --lr 1e-3 --score-act identity --epochs 4
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fedrec_with_pytorchdistributed_amd.config import FedRecConfig  # noqa: E402
from fedrec_with_pytorchdistributed_amd.data.sampler import validation_batches  # noqa: E402
from fedrec_with_pytorchdistributed_amd.data.synthetic import SynthSpec, SyntheticCorpus  # noqa: E402
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel  # noqa: E402
from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine  # noqa: E402


@torch.no_grad()
def diag(eng: LocalEngine, limit: int = 2048):
    V = eng.encode_all()
    m = eng.model
    m.eval()
    us, ss, mh_max, pool_max = [], [], [], []
    ue = m.user_encoder
    mha = ue.multihead_attention
    for cand_np, his_np in validation_batches(eng.shard.valid, 256, 4, 50, True, limit):
        cand, his = eng.to_device(cand_np), eng.to_device(his_np)
        B, C = cand.shape
        hv = V.index_select(0, his.reshape(-1).long()).view(B, his.shape[1], -1)
        cv = V.index_select(0, cand.reshape(-1).long()).view(B, C, -1)
        u = m.user_encoder(hv.float(), his)  # module path (the fused step returns no user vector)
        x = hv.float()
        q = torch.nn.functional.linear(x, mha.W_Q.weight, mha.W_Q.bias).view(B, -1, mha.n_heads, mha.d_k)
        k = torch.nn.functional.linear(x, mha.W_K.weight, mha.W_K.bias).view(B, -1, mha.n_heads, mha.d_k)
        sc = torch.einsum("bqhd,bkhd->bhqk", q, k) / mha.d_k ** 0.5
        mh_max.append(sc.amax(-1).flatten().cpu())
        y = mha(x)
        ad = ue.additive_attention
        a = torch.nn.functional.linear(torch.tanh(torch.nn.functional.linear(y, ad.att_fc1.weight, ad.att_fc1.bias)),
                                       ad.att_fc2.weight, ad.att_fc2.bias).squeeze(-1)
        pool_max.append(a.amax(-1).cpu())
        s = torch.bmm(cv, u.unsqueeze(-1)).squeeze(-1)
        us.append(u.norm(dim=-1).cpu())
        ss.append(s.cpu())
    S = torch.cat(ss)
    ties = float(((S.max(1).values - S.min(1).values).abs() < 1e-6).float().mean())
    fc = m.text_encoder.fc
    mh, pm = torch.cat(mh_max), torch.cat(pool_max)
    cliff = float(np.log(1e-8))
    return {"mhsa_rowmax_median": float(mh.median()), "mhsa_rows_below_cliff": float((mh < cliff).float().mean()),
            "mhsa_rows_zero": float((mh < -87.0).float().mean()), "pool_max_median": float(pm.median()),
            "pool_users_below_cliff": float((pm < cliff).float().mean()),
            "news_norm": float(V.norm(dim=1).mean()), "news_spread": float((V - V.mean(0)).norm(dim=1).mean()),
            "user_norm": float(torch.cat(us).mean()), "score_abs": float(S.abs().mean()),
            "score_spread": float((S.max(1).values - S.min(1).values).mean()), "tied_share": ties,
            "fc_w": float(fc.weight.norm()), "fc_b": float(fc.bias.norm())}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--score-act", default="identity")
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--preset", default="mind-small")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    cfg = FedRecConfig(mode="grad_avg", batch_size=64, lr=args.lr, score_act=args.score_act)
    torch.manual_seed(0)
    model = FedRecModel(cfg).to(dev)
    model.build_flat()
    shard = SyntheticCorpus(SynthSpec.preset(args.preset)).client_shard(0, 1)
    eng = LocalEngine(cfg, model, shard, dev)
    rows = [{"epoch": -1, **diag(eng)}]
    print(json.dumps(rows[-1]), flush=True)
    for ep in range(args.epochs):
        st = eng.train_epoch()
        va = eng.validate()
        rows.append({"epoch": ep, "train_loss": st["training_loss"], "valid_auc": va["valid_auc"],
                     "valid_mrr": va["valid_mrr"], **diag(eng), "args": vars(args)})
        print(json.dumps(rows[-1]), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
