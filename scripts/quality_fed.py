"""Federated quality at W > 1 on one GPU: GA, PA (K = 8) and star FedAvg with
W clients sharing the card (FEDREC_SHARE_GPU=1, gloo data plane), against the one-client run, on
the planted-signal synthetic shard -- the same impressions in every run (3 epochs / rounds over
the same users, split W ways) and the same impressions per optimizer step (per-client batch
64 / W), plain-CE scorer at lr 1e-4 (the reference's sigmoid-CE stays at
chance, docs/PARITY.md).  Every run's metrics JSONL is kept under ``--out``; a summary JSON line
per run goes to stdout.

    python scripts/quality_fed.py --out gpurun_out/quality_fed --world 4 8
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from launch_util import run_ranks  # noqa: E402

SHARE = {"FEDREC_CPU_ONLY": "0", "FEDREC_SHARE_GPU": "1", "FEDREC_DATA_BACKEND": "gloo", "FEDREC_QUIET": "1"}


def runs(world, epochs, preset):
    common = [f"--data_dir=synthetic:{preset}", "--lr=1e-4", "--score_act=identity", "--round_timeout_s=900",
              "--collective_timeout_s=900"]
    yield "ga_w1", [["Gradient_Averaging_main.py", str(epochs), "64", "0", *common]]
    for W in world:
        # equal work AND equal updates: W clients x batch 64 / W = the one-client run's 64
        # impressions per optimizer step (GA is then the same large-batch SGD, up to sampling)
        b = str(64 // W)
        yield f"ga_w{W}", [["Gradient_Averaging_main.py", str(epochs), b, "0", *common]] * W
        yield f"pa8_w{W}", [["Parameter_Averaging_main.py", str(epochs), b, "0", "--param_avg_every=8",
                             "--local_update=per_step", *common]] * W
        # star: per-step local Adam (the reference's client takes ONE optimizer step per local
        # epoch -- model.update() after the loop, client.py:100 -- which cannot learn in 3 rounds;
        # local_update=per_step is the schedule option that trains like the other modes)
        yield f"star_w{W}", ([["server.py", str(epochs), *common]] +
                             [["client.py", "1", b, "0", "0", "q", "--local_update=per_step", *common]] * W)
        # server-side step options (off by default): FedAvgM / server lr at the
        # coordinator, and for PA the clients' Adam moments averaged + the same server step
        for tag, extra in SERVER_VARIANTS:
            yield f"star_w{W}_{tag}", ([["server.py", str(epochs), *common, *extra]] +
                                       [["client.py", "1", b, "0", "0", "q", "--local_update=per_step", *common]] * W)
        for tag, extra in PA_VARIANTS:
            yield f"pa8_w{W}_{tag}", [["Parameter_Averaging_main.py", str(epochs), b, "0", "--param_avg_every=8",
                                       "--local_update=per_step", *common, *extra]] * W


SERVER_VARIANTS = [("m9", ["--server_momentum=0.9"]), ("lr3", ["--server_lr=3.0"]),
                   ("lr3m5", ["--server_lr=3.0", "--server_momentum=0.5"]),
                   ("adam1e2", ["--server_opt=adam", "--server_lr=0.01", "--server_momentum=0.9"]),
                   ("adam3e3", ["--server_opt=adam", "--server_lr=0.003", "--server_momentum=0.9"])]
PA_VARIANTS = [("mv", ["--pa_average_moments=1"]), ("mv_lr2", ["--pa_average_moments=1", "--server_lr=2.0"]),
               ("mv_m5", ["--pa_average_moments=1", "--server_momentum=0.5"]),
               ("mv_lr3", ["--pa_average_moments=1", "--server_lr=3.0"]),
               ("mv_lr2m5", ["--pa_average_moments=1", "--server_lr=2.0", "--server_momentum=0.5"]),
               ("mv_lr4", ["--pa_average_moments=1", "--server_lr=4.0"]),
               ("k4_mv_lr2", ["--pa_average_moments=1", "--server_lr=2.0", "--param_avg_every=4"])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/quality_fed")
    ap.add_argument("--world", type=int, nargs="+", default=[4, 8])
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--preset", default="small")
    ap.add_argument("--only", default="")
    ap.add_argument("--scratch", default="/tmp/quality_fed")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for name, argvs in runs(a.world, a.epochs, a.preset):
        # --only: comma list of substrings; a trailing "$" asks for the exact run name
        if a.only and not any((name == o[:-1]) if o.endswith("$") else (o in name) for o in a.only.split(",")):
            continue
        d = os.path.abspath(os.path.join(a.out, name))
        os.makedirs(d, exist_ok=True)
        mp = os.path.join(d, "metrics.jsonl")
        if os.path.exists(mp):
            os.remove(mp)
        # snapshots (270 MB with the frozen backbone) go to scratch, not beside the kept metrics
        sd = os.path.join(a.scratch, name)
        os.makedirs(sd, exist_ok=True)
        argvs = [[*v, f"--metrics_path={mp}", f"--snapshot_path={sd}/snapshot.pt", "--save_every=0"] for v in argvs]
        t0 = time.time()
        outs = run_ranks(argvs, SHARE, timeout=900, cwd=sd)
        dt = time.time() - t0
        ok = all(rc == 0 for rc, _ in outs)
        rec = {"run": name, "ok": ok, "wall_s": round(dt, 1), "processes": len(argvs)}
        if ok and os.path.exists(mp):
            rows = [json.loads(l) for l in open(mp) if l.strip()]
            fin = [r for r in rows if r.get("final_global")]
            rows = [r for r in rows if not r.get("final_global")]
            if fin:  # star: the final GLOBAL model's score (the per-round rows score local models)
                rec["global_valid_auc"] = round(fin[-1].get("global_valid_auc", float("nan")), 4)
                rec["global_valid_mrr"] = round(fin[-1].get("global_valid_mrr", float("nan")), 4)
            rec["valid_auc"] = [round(r.get("valid_auc", float("nan")), 4) for r in rows]
            rec["valid_mrr"] = [round(r.get("valid_mrr", float("nan")), 4) for r in rows]
            rec["training_loss"] = [round(r.get("training_loss", float("nan")), 4) for r in rows]
        else:
            rec["tail"] = "\n".join(o[-1500:] for _, o in outs)[-4000:]
        print(json.dumps(rec), flush=True)
        with open(os.path.join(a.out, "summary.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
