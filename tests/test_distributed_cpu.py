"""Multi-process runs of the three federation modes on CPU/gloo (BASELINE config 1), with the
reference's own launch contract (positional argv + RANK/WORLD_SIZE/MASTER_* env)."""
import json
import os

import pytest
import torch

from launch_util import ROOT, run_ranks

TINY = ["--data_dir=synthetic:tiny", "--backbone.name=tiny", "--round_timeout_s=120", "--collective_timeout_s=120"]


def _ok(outs):
    for rc, out in outs:
        assert rc == 0, out[-3000:]


def _metrics(path, final=False):
    """Per-round records (``final=True``: the star coordinator's final global-model record)."""
    with open(path) as f:
        rows = [json.loads(l) for l in f if l.strip()]
    return [r for r in rows if bool(r.get("final_global")) == final]


@pytest.mark.slow
def test_grad_avg_two_ranks(tmp_path):
    snap = str(tmp_path / "snapshot.pt")
    argv = ["Gradient_Averaging_main.py", "2", "16", "1", *TINY, f"--snapshot_path={snap}"]
    # TORCH_DISTRIBUTED_DEBUG=DETAIL: c10d wraps every process group in its collective checker
    # (op type, shapes and dtypes compared across ranks before each collective) -- a mismatched
    # collective sequence fails loudly here instead of hanging
    outs = run_ranks([argv, argv], {"FEDREC_DUMP_FLAT": str(tmp_path / "dump"), "TORCH_DISTRIBUTED_DEBUG": "DETAIL"})
    _ok(outs)
    a = torch.load(tmp_path / "dump" / "rank0.pt")
    b = torch.load(tmp_path / "dump" / "rank1.pt")
    assert torch.equal(a, b), "both encoders must stay synchronised (reference E5 diverges)"
    snapd = torch.load(snap, weights_only=True)
    assert set(snapd) >= {"MODEL_STATE", "EPOCHS_RUN"} and snapd["EPOCHS_RUN"] == 1
    assert len(snapd["MODEL_STATE"]) == 4 + 2 * 16 + 6 + 10
    m = _metrics(str(tmp_path / "metrics.jsonl"))
    assert len(m) == 2 and all(k in m[-1] for k in ("training_loss", "valid_auc", "val_ndcg@10"))


@pytest.mark.slow
@pytest.mark.parametrize("secure", [False, True])
def test_grad_avg_unfrozen_bucketed_two_ranks(tmp_path, secure):
    """Unfrozen backbone: gradients are reduced in buckets from autograd hooks during the
    backward (the DDP-reducer equivalent), plain or pairwise-masked; tiny buckets force many
    of them.  Both ranks must end bit-identical (GA keeps every client in lockstep)."""
    argv = ["Gradient_Averaging_main.py", "1", "16", "1", *TINY, "--backbone.frozen=0", "--backbone.dropout=0",
            "--backbone.attention_dropout=0",
            f"--secagg.enabled={int(secure)}", f"--snapshot_path={tmp_path}/s.pt"]
    outs = run_ranks([argv, argv], {"FEDREC_DUMP_FLAT": str(tmp_path / "dump"), "FEDREC_BUCKET_MB": "0.05",
                                    "FEDREC_COLL_CHECK": "1"})
    _ok(outs)
    a = torch.load(tmp_path / "dump" / "rank0.pt")
    b = torch.load(tmp_path / "dump" / "rank1.pt")
    assert a.numel() > 2_000_000  # the backbone is in the trainable set
    assert torch.equal(a, b)


@pytest.mark.slow
def test_bucketed_reducer_matches_flat_allreduce(tmp_path):
    """The backward-overlapped bucket reducer must reduce exactly what the flat all-reduce of
    the whole gradient reduces: same buckets summed once, scale 1/W, every bucket after all of
    its gradients landed.  Lockstep alone (both ranks equal) would not catch a skipped or early
    bucket; the unbucketed run is the oracle.  (The pairwise-masked op is pinned per bucket by
    test_bucket_reducer_sums_match_flat_oracle: its fixed-point grid follows each bucket's own
    bound, so whole runs differ by grid steps that Adam amplifies on near-zero coordinates.)"""
    base = ["Gradient_Averaging_main.py", "1", "16", "0", *TINY, "--backbone.frozen=0", "--backbone.dropout=0",
            "--backbone.attention_dropout=0"]
    flat = base + ["--bucket_reducer=0"]
    _ok(run_ranks([flat, flat], {"FEDREC_DUMP_FLAT": str(tmp_path / "flat")}))
    _ok(run_ranks([base, base], {"FEDREC_DUMP_FLAT": str(tmp_path / "buck"), "FEDREC_BUCKET_MB": "0.05"}))
    a = torch.load(tmp_path / "flat" / "rank0.pt")
    b = torch.load(tmp_path / "buck" / "rank0.pt")
    assert torch.equal(b, torch.load(tmp_path / "buck" / "rank1.pt"))
    assert float((a - b).abs().max()) <= 1e-7, float((a - b).abs().max())


@pytest.mark.slow
def test_secure_sum_exact_eight_clients():
    """Secure aggregation at W = 8 (BASELINE config 5's client count): the masked sum equals
    the plain sum within the fixed-point grid at every step -- an all-zero first step, single-
    client largest coordinates with the holder alternating and a 10x jump per step, cancelling
    opposite signs, tiny values -- so no coordinate is ever clamped; a non-finite value on one
    client makes the result NaN."""
    outs = run_ranks([["tests/_secagg_worker.py"]] * 8, timeout=180)
    _ok(outs)
    for _, out in outs:
        assert "SECAGG OK" in out, out[-2000:]


@pytest.mark.slow
def test_bucket_reducer_sums_match_flat_oracle():
    """Reducer-level oracle: per bucket, the reduced gradient equals an explicit flat SUM
    all-reduce of every rank's gradient -- exactly for op=mean, within the bucket's fixed-point
    grid for op=secure -- over gradients spanning 8 decades and several steps."""
    outs = run_ranks([["tests/_reducer_worker.py"]] * 2, timeout=120)
    _ok(outs)
    for _, out in outs:
        assert "REDUCER OK" in out, out[-2000:]


@pytest.mark.slow
def test_grad_avg_per_epoch_unfrozen_two_ranks(tmp_path):
    """grad_avg with the per-epoch schedule and an unfrozen backbone: the bucket reducer is
    installed but no backward arms it (several accumulated batches, one epoch-end step), so
    finish() must reduce every bucket itself."""
    argv = ["Gradient_Averaging_main.py", "1", "8", "0", *TINY, "--backbone.frozen=0", "--backbone.dropout=0",
            "--backbone.attention_dropout=0", "--local_update=per_epoch"]
    _ok(run_ranks([argv, argv], {"FEDREC_DUMP_FLAT": str(tmp_path / "dump"), "FEDREC_BUCKET_MB": "0.05"}))
    a = torch.load(tmp_path / "dump" / "rank0.pt")
    assert torch.equal(a, torch.load(tmp_path / "dump" / "rank1.pt"))


@pytest.mark.slow
def test_param_avg_two_ranks(tmp_path):
    argv = ["Parameter_Averaging_main.py", "2", "16", "1", *TINY, f"--snapshot_path={tmp_path}/s.pt"]
    outs = run_ranks([argv, argv], {"FEDREC_DUMP_FLAT": str(tmp_path / "dump")})
    _ok(outs)
    a = torch.load(tmp_path / "dump" / "rank0.pt")
    b = torch.load(tmp_path / "dump" / "rank1.pt")
    assert torch.allclose(a, b, atol=1e-6), "parameters are averaged after every epoch"


@pytest.mark.slow
def test_param_avg_every_k_steps(tmp_path):
    argv = ["Parameter_Averaging_main.py", "1", "8", "1", *TINY, "--local_update=per_step", "--param_avg_every=3",
            f"--snapshot_path={tmp_path}/s.pt"]
    _ok(run_ranks([argv, argv], {"FEDREC_DUMP_FLAT": str(tmp_path / "dump")}))


@pytest.mark.slow
def test_star_fedavg_server_plus_two_clients(tmp_path):
    snap = str(tmp_path / "server_snapshot.pt")
    server = ["server.py", "2", *TINY, f"--snapshot_path={snap}", "--round_artifacts=1"]
    client = ["client.py", "1", "16", "1", "0", "c", *TINY, f"--snapshot_path={tmp_path}/c.pt", "--round_artifacts=1"]
    # the coordinator is rank 1 here on purpose: roles come from the entrypoint (Q13)
    outs = run_ranks([client, server, client], {"FEDREC_DUMP_FLAT": str(tmp_path / "dump"),
                                                "FEDREC_STAR_AGG": "upload"})
    _ok(outs)
    hist = _metrics(str(tmp_path / "metrics.jsonl"))
    assert [h["round"] for h in hist] == [0, 1] and all(h["clients_accepted"] == 2 for h in hist)
    # after the last round the clients score the final GLOBAL model (the per-round rows score
    # their local models, as the reference's client-side validate does)
    fin = _metrics(str(tmp_path / "metrics.jsonl"), final=True)
    assert len(fin) == 1 and fin[0]["clients_reporting"] == 2 and 0.0 <= fin[0]["global_valid_auc"] <= 1.0, fin
    assert os.path.exists(tmp_path / "global_model_round1.pt")
    g = torch.load(tmp_path / "global_model_round1.pt", weights_only=True)
    snapd = torch.load(snap, weights_only=True)
    assert snapd["ROUND"] == 1
    # reference interchange files: each client's model.pt (client.py:288) and the server's
    # received_model_{k}.pt (server.py:27); the global model is their unweighted mean
    # (server.py:46-50) -- all in the 116-key reference state_dict layout
    r0 = torch.load(tmp_path / "received_model_0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "received_model_1.pt", weights_only=True)
    m0 = torch.load(tmp_path / "client0" / "model.pt", weights_only=True)
    assert set(r0) == set(g) == set(m0)
    for key in ("text_encoder.fc.weight", "user_encoder.additive_attention.att_fc1.weight"):
        assert torch.allclose(g[key], (r0[key] + r1[key]) / 2, atol=1e-6), key
    assert not torch.equal(r0["text_encoder.fc.weight"], r1["text_encoder.fc.weight"])
    # model sync: client 0 read the global model once and broadcast it over the client data group
    assert "model sync: {'backend': 'gloo', 'size': 2}" in outs[0][1] + outs[2][1]
    # every client kept its own resumable snapshot (Adam moments + step, RNG, engine counters)
    for k in (0, 1):
        cs = torch.load(tmp_path / f"client{k}_c.pt", weights_only=True)
        assert cs["ROUND"] == 1 and int(cs["OPTIM_STATE"]["step"]) == 2 and "RNG" in cs and "ENGINE" in cs


def test_server_step_math():
    """ServerStep: identity at the defaults (the reference's plain mean); FedAvgM + server lr:
    v_r = beta v_{r-1} + (avg_r - theta_r), theta_{r+1} = theta_r + lr v_r."""
    from fedrec_with_pytorchdistributed_amd.train.federated import ServerStep
    s0 = ServerStep()
    th, avg = torch.randn(10), torch.randn(10)
    assert not s0.active and s0.apply(th, avg) is avg and s0.state() is None
    s = ServerStep(lr=1.5, momentum=0.9)
    th0 = torch.zeros(10, dtype=torch.float64)
    a0, a1 = torch.randn(10, dtype=torch.float64), torch.randn(10, dtype=torch.float64)
    th1 = s.apply(th0, a0)
    assert torch.allclose(th1, 1.5 * a0)
    th2 = s.apply(th1, a1)
    v = 0.9 * a0 + (a1 - th1)
    assert torch.allclose(th2, th1 + 1.5 * v)
    s2 = ServerStep(lr=1.5, momentum=0.9)
    s2.load(s.state())  # resume carries the momentum
    assert torch.equal(s2.v, s.v)
    # FedAdam: m = b1 m + (1 - b1) d, v = b2 v + (1 - b2) d^2, theta = theta_g + lr m / (sqrt(v) + tau)
    fa = ServerStep(lr=0.01, momentum=0.9, opt="adam", beta2=0.99, tau=1e-3)
    t1 = fa.apply(th0, a0)
    m1, v1 = 0.1 * a0, 0.01 * a0 * a0
    assert torch.allclose(t1, th0 + 0.01 * m1 / (v1.sqrt() + 1e-3))
    t2 = fa.apply(t1, a1)
    d1 = a1 - t1
    m2, v2 = 0.9 * m1 + 0.1 * d1, 0.99 * v1 + 0.01 * d1 * d1
    assert torch.allclose(t2, t1 + 0.01 * m2 / (v2.sqrt() + 1e-3))
    fb = ServerStep(opt="adam")
    fb.load(fa.state())
    assert torch.equal(fb.s, fa.s) and torch.equal(fb.v, fa.v)


@pytest.mark.slow
def test_star_server_learning_rate(tmp_path):
    """The coordinator's server step (cfg.server_lr): global_{r+1} = global_r + lr (mean_r -
    global_r), checked from the clients' round-1 uploads (received_model_k.pt) and the saved
    global models; the snapshot carries the server step's buffer for a resume."""
    snap = str(tmp_path / "server_snapshot.pt")
    server = ["server.py", "2", *TINY, f"--snapshot_path={snap}", "--round_artifacts=1", "--server_lr=2.0"]
    client = ["client.py", "1", "16", "1", "0", "c", *TINY, f"--snapshot_path={tmp_path}/c.pt", "--round_artifacts=1"]
    _ok(run_ranks([server, client, client], {"FEDREC_STAR_AGG": "upload"}))
    g0 = torch.load(tmp_path / "global_model_round0.pt", weights_only=True)
    g1 = torch.load(tmp_path / "global_model_round1.pt", weights_only=True)
    r0 = torch.load(tmp_path / "received_model_0.pt", weights_only=True)  # round 1's uploads
    r1 = torch.load(tmp_path / "received_model_1.pt", weights_only=True)
    for key in ("text_encoder.fc.weight", "user_encoder.additive_attention.att_fc1.weight"):
        mean1 = (r0[key].double() + r1[key].double()) / 2
        want = (g0[key].double() + 2.0 * (mean1 - g0[key].double())).float()
        assert torch.allclose(g1[key], want, atol=1e-6), key
        if float((mean1 - g0[key].double()).abs().max()) > 1e-5:  # (a key that moved this round)
            assert not torch.allclose(g1[key], mean1.float(), atol=1e-6), key
    sd = torch.load(snap, weights_only=True)
    assert "SERVER_OPT" in sd and sd["SERVER_OPT"]["v"].dtype == torch.float64


@pytest.mark.slow
def test_param_avg_moments_and_server_momentum(tmp_path):
    """PA with the clients' Adam moments averaged and a server step on the mean: every client
    applies it to the same all-reduced inputs, so the clients stay bitwise identical; the
    trajectory differs from the plain mean's."""
    base = ["Parameter_Averaging_main.py", "2", "8", "1", *TINY, "--local_update=per_step", "--param_avg_every=2"]
    opt = base + ["--pa_average_moments=1", "--server_momentum=0.9", "--server_lr=1.5",
                  f"--snapshot_path={tmp_path}/s.pt"]
    _ok(run_ranks([opt, opt], {"FEDREC_DUMP_FLAT": str(tmp_path / "opt")}))
    _ok(run_ranks([base + [f"--snapshot_path={tmp_path}/b.pt"]] * 2, {"FEDREC_DUMP_FLAT": str(tmp_path / "base")}))
    a = torch.load(tmp_path / "opt" / "rank0.pt")
    assert torch.equal(a, torch.load(tmp_path / "opt" / "rank1.pt"))
    assert not torch.equal(a, torch.load(tmp_path / "base" / "rank0.pt"))
    sd = torch.load(tmp_path / "s.pt", weights_only=True)
    assert "SERVER_OPT" in sd


@pytest.mark.slow
def test_star_fedavg_allreduce_aggregation(tmp_path):
    server = ["server.py", "2", *TINY, f"--snapshot_path={tmp_path}/s.pt"]
    client = ["client.py", "1", "16", "1", "0", "c", *TINY]
    outs = run_ranks([server, client, client], {"FEDREC_STAR_AGG": "allreduce"})
    _ok(outs)


@pytest.mark.slow
def test_star_quorum_survives_killed_client(tmp_path):
    server = ["server.py", "2", *TINY, "--quorum=0.5", "--round_timeout_s=25", f"--snapshot_path={tmp_path}/s.pt"]
    client = ["client.py", "1", "16", "1", "0", "c", *TINY, "--quorum=0.5", "--round_timeout_s=60"]
    outs = run_ranks([server, client, client], {"FEDREC_FAULT": "client:1:round:1:kill"}, timeout=200)
    assert outs[0][0] == 0, outs[0][1][-3000:]
    hist = _metrics(str(tmp_path / "metrics.jsonl"))
    assert [h["clients_accepted"] for h in hist] == [2, 1]


@pytest.mark.slow
def test_star_heartbeat_detects_killed_client_early(tmp_path):
    """A killed client stops heartbeating: with a 10-minute round timeout the coordinator
    still closes the round after heartbeat_timeout_s (quorum 0.5) and logs it dead."""
    import time as _t
    hb = ["--quorum=0.5", "--round_timeout_s=600", "--heartbeat_timeout_s=8", "--heartbeat_s=0.5"]
    server = ["server.py", "2", *TINY, *hb, f"--snapshot_path={tmp_path}/s.pt"]
    client = ["client.py", "1", "16", "1", "0", "c", *TINY, *hb]
    t0 = _t.monotonic()
    outs = run_ranks([server, client, client], {"FEDREC_FAULT": "client:1:round:1:kill"}, timeout=300)
    assert outs[0][0] == 0, outs[0][1][-3000:]
    assert _t.monotonic() - t0 < 240
    hist = _metrics(str(tmp_path / "metrics.jsonl"))
    assert [h["clients_accepted"] for h in hist] == [2, 1]
    assert hist[1]["clients_dead"] == [1]


@pytest.mark.slow
def test_star_rejects_nan_upload(tmp_path):
    server = ["server.py", "1", *TINY, "--quorum=0.5", "--round_timeout_s=60", f"--snapshot_path={tmp_path}/s.pt"]
    client = ["client.py", "1", "16", "1", "0", "c", *TINY, "--quorum=0.5"]
    outs = run_ranks([server, client, client], {"FEDREC_FAULT": "client:0:round:0:nan"})
    _ok(outs)
    hist = _metrics(str(tmp_path / "metrics.jsonl"))
    assert hist[0]["clients_accepted"] == 1
    g = torch.load(tmp_path / "global_model_round0.pt", weights_only=True)
    assert all(torch.isfinite(v).all() for v in g.values())


def _star_round0(tmp_path, tag, weighted, secure, W=4):
    """One star round (1 coordinator + W clients, tiny shards); returns (global after round 0,
    every client's final parameters, the round-0 global broadcast) -- clients train exactly one
    round, so their dumped parameters are what they uploaded."""
    d = tmp_path / tag
    flags = [f"--weighted_fedavg={int(weighted)}", f"--secagg.enabled={int(secure)}"]
    server = ["server.py", "1", *TINY, *flags, f"--snapshot_path={d}/s.pt"]
    client = ["client.py", "1", "16", "1", "0", "c", *TINY, *flags]
    outs = run_ranks([server] + [client] * W, {"FEDREC_DUMP_FLAT": str(d / "dump"), "FEDREC_STAR_AGG": "upload"},
                     timeout=300)
    _ok(outs)
    g = torch.load(d / "global_model_round0.pt", weights_only=True)
    cl = [torch.load(d / "dump" / f"rank{i}.pt") for i in range(1, W + 1)]
    return g, cl, outs


@pytest.mark.slow
@pytest.mark.parametrize("weighted", [False, True])
def test_star_secure_aggregation_is_the_plain_mean(tmp_path, weighted):
    """Secure aggregation in the star mode (1 coordinator + 4 clients): the clients upload their
    WEIGHTED model deltas on the fixed-point grid a masked exponent histogram agrees
    (parallel.secagg.StarSecureUpload), so the coordinator's global model is the plain
    (weighted) FedAvg mean of the client models -- server.py:46-50 -- to fp32 rounding; nothing
    is clamped.  The same round without secure aggregation gives the same global model, and the
    weighted mean differs from the unweighted one (the shards differ in size)."""
    from fedrec_with_pytorchdistributed_amd.config import BackboneConfig, FedRecConfig
    from fedrec_with_pytorchdistributed_amd.data.synthetic import SynthSpec, SyntheticCorpus
    from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel

    gs, cs, _ = _star_round0(tmp_path, "secure", weighted, True)
    gp, cp_, _ = _star_round0(tmp_path, "plain", weighted, False)
    W = len(cs)
    corpus = SyntheticCorpus(SynthSpec.preset("tiny"))
    n = [len(corpus.client_shard(k, W).train) for k in range(W)]
    w = torch.tensor([float(x) if weighted else 1.0 for x in n], dtype=torch.float64)
    cfg = FedRecConfig()
    cfg.backbone = BackboneConfig.preset("tiny")
    fl = FedRecModel(cfg).build_flat()
    for name, p, off in fl.views():
        sl = slice(off, off + p.numel())
        mean = sum(wk * c[sl].double() for wk, c in zip(w, cs)) / w.sum()
        assert torch.allclose(gs[name].reshape(-1).double(), mean, atol=2e-6, rtol=0), name
        mean_p = sum(wk * c[sl].double() for wk, c in zip(w, cp_)) / w.sum()
        assert torch.allclose(gp[name].reshape(-1).double(), mean_p, atol=2e-6, rtol=0), name
    # the two runs trained the same clients from the same start: same uploads, same global model
    for a, b in zip(cs, cp_):
        assert torch.equal(a, b)
    for k in gs:
        assert torch.allclose(gs[k], gp[k], atol=2e-6, rtol=0), k
    if weighted:
        assert len(set(n)) > 1


@pytest.mark.slow
def test_grad_avg_resume_from_snapshot(tmp_path):
    snap = str(tmp_path / "snapshot.pt")
    argv = ["Gradient_Averaging_main.py", "1", "16", "1", *TINY, f"--snapshot_path={snap}"]
    _ok(run_ranks([argv, argv]))
    s1 = torch.load(snap, weights_only=True)
    argv2 = ["Gradient_Averaging_main.py", "2", "16", "1", *TINY, f"--snapshot_path={snap}"]
    outs = run_ranks([argv2, argv2])
    _ok(outs)
    assert "resuming" in outs[0][1]
    s2 = torch.load(snap, weights_only=True)
    assert s1["EPOCHS_RUN"] == 0 and s2["EPOCHS_RUN"] == 1


@pytest.mark.slow
def test_grad_avg_secure_aggregation_matches_plain(tmp_path):
    """Masked int32 all-reduce of the gradients == plain averaging up to the fixed-point step."""
    base = ["Gradient_Averaging_main.py", "1", "16", "1", *TINY, "--save_every=0"]
    _ok(run_ranks([base, base], {"FEDREC_DUMP_FLAT": str(tmp_path / "plain")}))
    sec = base + ["--secagg.enabled=1"]
    _ok(run_ranks([sec, sec], {"FEDREC_DUMP_FLAT": str(tmp_path / "sec")}))
    a = torch.load(tmp_path / "plain" / "rank0.pt")
    b = torch.load(tmp_path / "sec" / "rank0.pt")
    c = torch.load(tmp_path / "sec" / "rank1.pt")
    assert torch.equal(b, c)
    # Adam normalises each coordinate, so a gradient near the fixed-point step can move its
    # parameter by up to lr per step either way: bound the bulk tightly, the tail by lr * steps
    # (the running bound -- 4x the previous public mean's max, so no per-step MAX collective --
    # puts the grid ~2 bits coarser than an exact per-step max|g| would)
    d = (a - b).abs()
    assert float(torch.quantile(d.float(), 0.999)) < 4e-6
    assert float((d > 1e-6).float().mean()) < 4e-3
    assert float(d.max()) < 5e-5 * 40  # lr x (an upper bound on the epoch's steps)


@pytest.mark.slow
@pytest.mark.parametrize("config", [2, 3, 4])
def test_bench_contract_two_ranks(config):
    """bench.py under the driver's multi-rank launch contract (gloo here, RCCL on the node):
    exactly one JSON line, from rank 0, with the whole-job value and the BASELINE metric."""
    argv = ["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "4", "--preset", "tiny",
            "--backbone", "tiny", "--config", str(config), "--pa-every", "1", "--valid-limit", "16"]
    outs = run_ranks([argv, argv], timeout=300)
    _ok(outs)
    lines = [[l for l in out.splitlines() if l.startswith("{")] for _, out in outs]
    assert len(lines[0]) == 1 and lines[1] == []
    r = json.loads(lines[0][0])
    assert r["metric"].startswith("impressions/sec/node") and r["n_gpus"] == 2 and r["steps"] == 2
    assert r["config"]["global_batch"] == 8 and r["config"]["parallelism"] == "dp2"
    assert abs(r["value"] - 8 * 2 / (r["ms_per_step"] * 2 / 1000)) / r["value"] < 0.01
    assert r["scaling"] == "weak" and r["higher_is_better"] is True


@pytest.mark.slow
def test_allreduce_sweep_two_ranks():
    argv = ["benchmarks/allreduce_bench.py", "--max-mb", "0.1", "--iters", "2", "--warmup", "1"]
    outs = run_ranks([argv, argv], timeout=120)
    _ok(outs)
    rows = [json.loads(l) for l in outs[0][1].splitlines() if l.startswith("{")]
    assert rows and all(r["world"] == 2 and r["us"] > 0 for r in rows)


@pytest.mark.slow
@pytest.mark.parametrize("diverge", [False, True])
def test_collective_checker_two_ranks(diverge):
    """SURVEY §5.2 collective-sequence checker: identical sequences pass; a rank that issues a
    bucket with another reduction is reported on every rank with the first differing collective."""
    argv = ["tests/_collcheck_worker.py"] + (["--diverge"] if diverge else [])
    outs = run_ranks([argv, argv], {"FEDREC_COLL_CHECK": "1"}, timeout=120)
    _ok(outs)
    for _, out in outs:
        line = [l for l in out.splitlines() if l.startswith("COLLCHECK")][0]
        if not diverge:
            assert line == "COLLCHECK OK 5"
        else:
            assert "MISMATCH" in line and "first difference at collective #4" in line
            assert "all_reduce|float32|8|SUM" in line and "all_reduce|float32|8|MAX" in line


@pytest.mark.slow
def test_grad_avg_with_collective_checker(tmp_path):
    """The real GA / PA call sites under FEDREC_COLL_CHECK=1: the per-epoch verification passes."""
    snap = str(tmp_path / "snapshot.pt")
    for script in ("Gradient_Averaging_main.py", "Parameter_Averaging_main.py"):
        argv = [script, "2", "16", "1", *TINY, f"--snapshot_path={snap}"]
        outs = run_ranks([argv, argv], {"FEDREC_COLL_CHECK": "1"})
        _ok(outs)


def test_single_process_context_is_one_client(monkeypatch):
    """world == 1 (the bench's N=1 path): a one-client context with no process groups."""
    from fedrec_with_pytorchdistributed_amd.parallel import dist as fdist
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ctx = fdist.init(device="cpu")
    assert ctx.world == 1 and ctx.num_clients == 1 and ctx.client_index == 0 and not ctx.initialized
    assert ctx.client_ctrl_group is None and ctx.data_group is None
    assert fdist.make_grad_allreduce(ctx) is None or callable(fdist.make_grad_allreduce(ctx))


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4])
def test_cooperative_cache_matches_local_build(world):
    """Cooperative catalog encode (parallel/catalog.py): W clients each encode 1/W of the
    union of their news tables, all-gather the shares over the data plane, and place their own
    rows; every client's table equals the one it builds alone, bitwise, and every catalog title
    is encoded exactly once (several gather pieces, uneven shares)."""
    outs = run_ranks([["tests/_catalog_worker.py"]] * world, timeout=240)
    _ok(outs)
    for _, out in outs:
        assert "CATALOG OK 0.0" in out, out[-2000:]


@pytest.mark.parametrize("what", ["backbone", "tokens"])
def test_cooperative_cache_refuses_divergent_clients(what):
    """VERDICT r5 item 5 / ADVICE r5: a client whose frozen backbone differs by ONE weight, or
    whose token row of a shared title differs, must not silently receive the others' hidden
    states -- every client falls back to its own local build (attach returns None, with the
    reason), and they all agree on it (no client left waiting in the gather)."""
    outs = run_ranks([["tests/_catalog_worker.py", "--perturb", what]] * 2, timeout=240)
    _ok(outs)
    for _, out in outs:
        assert "CATALOG REFUSED" in out, out[-2000:]
        assert ("backbone" in out) if what == "backbone" else ("token rows" in out), out[-2000:]


def test_catalog_ids_and_hashes():
    """Leading zeros do not alias a catalog id; token-row hashes tell rows apart; the
    transient size counts a ring of pieces, not the union."""
    import numpy as np

    from fedrec_with_pytorchdistributed_amd.parallel import catalog
    g = catalog.global_ids(["<unk>", "N123", "N0123", "N0"])
    assert g[0] == -1 and g[1] == 123 and g[2] < -1 and g[3] == 0
    tok = torch.zeros(4, 2, 6, dtype=torch.int32)
    tok[1, 0, :3] = torch.tensor([101, 7, 102])
    tok[2] = tok[1]
    tok[3] = tok[1]
    tok[3, 1, 0] = 1
    h = catalog.token_row_hashes(tok)
    assert h[1] == h[2] and len({int(h[0]), int(h[1]), int(h[3])}) == 3
    with pytest.raises(catalog.CatalogMismatch):
        catalog._check_token_hashes([np.array([5, 6]), np.array([6, 7])], [np.array([1, 2]), np.array([3, 4])])
    catalog._check_token_hashes([np.array([5, 6]), np.array([6, 7])], [np.array([1, 2]), np.array([2, 4])])
    plan = catalog.CatalogPlan(0, 8, 8000, np.zeros(0, np.int64), np.zeros(0, np.int64), 4, 2000, 64000)
    assert catalog.transient_bytes(plan, 50, 768, 2) == 50 * 768 * 2 * 2000 * (2 * 8 + 2 + 8)


@pytest.mark.slow
def test_grad_avg_cooperative_cache_same_trajectory(tmp_path):
    """GA with the hidden-state cache on: the cooperative build (default at W > 1) and per-client
    builds (FEDREC_COOP_CACHE=0) give bit-identical final parameters."""
    argv = ["Gradient_Averaging_main.py", "1", "16", "0", *TINY, "--news_cache=hidden"]
    _ok(run_ranks([argv, argv], {"FEDREC_DUMP_FLAT": str(tmp_path / "coop")}))
    _ok(run_ranks([argv, argv], {"FEDREC_DUMP_FLAT": str(tmp_path / "local"), "FEDREC_COOP_CACHE": "0"}))
    a = torch.load(tmp_path / "coop" / "rank0.pt")
    assert torch.equal(a, torch.load(tmp_path / "coop" / "rank1.pt"))
    assert torch.equal(a, torch.load(tmp_path / "local" / "rank0.pt"))
