"""Typed configuration for the federated news-recommendation engine.

Every hard-coded constant of the reference is a field here:

* npratio / max_his_len          -> reference ``dataset.py:8-9``
* news_dim 400                   -> ``encoder.py:14,38``; ``client.py:33,35``
* user heads / d_k / query dim   -> ``encoder.py:39-47``
* text additive hidden 768 // 2  -> ``encoder.py:20-21``
* user dropout 0.2               -> ``encoder.py:43,50``
* lr 5e-5 (both Adams)           -> ``model.py:22-23``
* DP C=2, delta=1e-5, epochs=50  -> ``client.py:220-223``
* snapshot path / data dir       -> ``client.py:213,229``

Values are overridable with ``--key=value`` flags (dotted keys reach the nested
sections, e.g. ``--dp.epsilon=10``).  The reference's positional argv contract is
handled by the entrypoint shims (``client.py`` etc.), which build a config and then
apply any trailing ``--key=value`` overrides.

Behavioural quirks of the reference are individual switches in
:class:`Compat`; ``--compat.reference_quirks=1`` turns all of them on at once.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional


@dataclass
class BackboneConfig:
    """Transformer text backbone.  Defaults = ``distilbert-base-uncased`` config (E2)."""

    name: str = "distilbert"  # distilbert | bert-base
    vocab_size: int = 30522
    dim: int = 768
    n_layers: int = 6
    n_heads: int = 12
    hidden_dim: int = 3072
    max_position: int = 512
    ln_eps: float = 1e-12
    # HF DistilBERT train-mode dropout (Philox counter masks, ops.dropout_add / title attention):
    # `dropout` after the embedding LayerNorm and after FFN lin2, `attention_dropout` on the
    # attention probabilities.  Active in the unfrozen training forward (config 5) and in the
    # reference-compat train-mode replay (Q4); the frozen backbone's vectors are eval-mode
    # (model.py:42), so its hidden-state cache never sees dropout.
    dropout: float = 0.1
    attention_dropout: float = 0.1
    frozen: bool = True  # reference freezes DistilBERT (model.py:25-26)
    init_std: float = 0.02
    # local Hugging Face checkpoint (directory from save_pretrained, or one weights file) of
    # DistilBERT / BERT; "" = random init (no pretrained weights ship offline)
    pretrained: str = ""

    @staticmethod
    def preset(name: str) -> "BackboneConfig":
        if name in ("distilbert", "distilbert-base-uncased"):
            return BackboneConfig(name="distilbert")
        if name in ("bert-base", "bert-base-uncased"):
            # BASELINE config 5: unfrozen BERT-base text encoder (12 layers, same widths).
            return BackboneConfig(name="bert-base", n_layers=12, frozen=False)
        if name == "tiny":  # test-only preset
            return BackboneConfig(name="tiny", vocab_size=30522, dim=64, n_layers=2,
                                  n_heads=4, hidden_dim=128)
        raise ValueError(f"unknown backbone preset {name!r}")


@dataclass
class DPConfig:
    """Local differential privacy on per-occurrence news-vector gradients (client.py:87-89)."""

    enabled: bool = False
    epsilon: float = 0.0
    delta: float = 1e-5
    clip: float = 2.0  # MAX_GRAD_NORM (client.py:220)
    epochs: int = 50  # EPOCHS used for calibration (client.py:223)
    noise_multiplier: Optional[float] = None  # explicit sigma overrides calibration


@dataclass
class SecAggConfig:
    """Pairwise-mask secure aggregation (README.md:56,65 describes it; never implemented there)."""

    enabled: bool = False
    # no grid settings: every secure sum agrees its fixed-point bound through a masked exponent
    # histogram (gradients: parallel.secagg.ExactMasker; star uploads: StarSecureUpload, which
    # quantises the weighted model delta), so no coordinate is ever clamped


@dataclass
class Compat:
    """Switches that reproduce reference quirks.  All default to the fixed behaviour."""

    reference_quirks: bool = False  # master switch: turns every switch below on
    grad_double_last_batch: bool = False  # Q2: user grads x2, last batch only
    replay_train_mode: bool = False  # Q4: epoch-end replay re-runs the backbone with dropout
    no_history_truncation: bool = False  # Q6: pad to 50 but never truncate
    ldp_no_clip: bool = False  # Q10: no clip, noise std = sigma (not sigma*C)
    resplit_shard: bool = False  # Q11: DistributedSampler re-splits the private shard
    validate_last_only: bool = False  # Q9: report the last impression's metrics

    def resolved(self) -> "Compat":
        if not self.reference_quirks:
            return self
        return Compat(True, True, True, True, True, True, True)


@dataclass
class FedRecConfig:
    # --- model (encoder.py / attention.py) -------------------------------------------
    news_dim: int = 400
    user_heads: int = 20
    user_head_dim: int = 20
    user_query_dim: int = 200
    user_dropout: float = 0.2
    text_query_dim: int = 0  # 0 = backbone dim // 2 = 384 for DistilBERT (encoder.py:20-21)
    title_len: int = 50
    backbone: BackboneConfig = field(default_factory=BackboneConfig)
    score_act: str = "sigmoid"  # Q1: CE over sigmoid scores (model.py:123); "identity" optional
    mask_padding: bool = False  # Q7: reference never masks padding in pools/user MHA

    # --- data (dataset.py) -----------------------------------------------------------
    npratio: int = 4
    max_his_len: int = 50
    data_dir: str = "UserData"

    # --- optimisation (model.py:22-23) -----------------------------------------------
    lr: float = 5e-5
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_eps: float = 1e-8
    batch_size: int = 16
    total_epochs: int = 1
    save_every: int = 1  # GA / PA snapshots every N epochs; star-mode CLIENT snapshots are written every round
    global_rounds: int = 1

    # --- federation ------------------------------------------------------------------
    # fedavg_star | grad_avg | param_avg (main.py, "every participant trains", is grad_avg)
    mode: str = "fedavg_star"
    local_update: str = "auto"  # per_epoch | per_step | auto (per_step for grad_avg)
    param_avg_every: int = 0  # PA: all-reduce every K local steps (0 = once per epoch)
    weighted_fedavg: bool = False  # Q12: reference mean is unweighted (server.py:49)
    # server-side step on the averaged update (defaults = the reference's plain mean,
    # server.py:46-50 / Parameter_Averaging_main.py:144-148): the new global model is
    # theta_g + server_lr * v, v = server_momentum * v + (mean_k theta_k - theta_g) -- FedAvgM
    # (Hsu et al. 2019) with a server learning rate (Reddi et al. 2021).  Star: at the
    # coordinator; PA: on every client, identically (the same inputs give bitwise-same models)
    server_lr: float = 1.0
    server_momentum: float = 0.0
    # "sgd": the step above; "adam": FedAdam (Reddi et al. 2021) on the pseudo-gradient
    # d = mean_k theta_k - theta_g: m = momentum m + (1 - momentum) d, v = beta2 v + (1 - beta2)
    # d^2, theta = theta_g + server_lr m / (sqrt(v) + tau)
    server_opt: str = "sgd"
    server_beta2: float = 0.99
    server_tau: float = 1e-3
    pa_average_moments: bool = False  # PA: average the clients' Adam m / v with the parameters
    # unfrozen backbone (GA): reduce the gradient in ~28 MB buckets during the backward (DDP's
    # reducer, parallel/reducer.py); False = one flat all-reduce after it
    bucket_reducer: bool = True
    sync: str = "trainable"  # Q15: trainable | full (the reference syncs all 116 tensors)
    quorum: float = 1.0  # fraction of clients needed to aggregate a round
    collective_timeout_s: float = 600.0  # reference: 2 days (client.py:227)
    round_timeout_s: float = 3600.0
    # star-mode liveness: clients bump a progress counter in the store at most
    # every heartbeat_s (per training step, around validation and upload); the coordinator
    # declares a client dead when its counter has not moved for heartbeat_timeout_s (0 = off)
    # and aggregates the quorum without waiting out round_timeout_s
    heartbeat_s: float = 2.0
    heartbeat_timeout_s: float = 300.0

    # --- privacy / secure aggregation --------------------------------------------------
    dp: DPConfig = field(default_factory=DPConfig)
    secagg: SecAggConfig = field(default_factory=SecAggConfig)

    # --- engine ------------------------------------------------------------------------
    precision: str = "bf16"  # backbone compute dtype: bf16 | fp32
    # HBM-resident cache of the frozen backbone's hidden states [N, T, D]:
    # auto = on for a frozen backbone on the device when the table fits in a quarter of the
    # free HBM; hidden = always (also on the host); none = re-encode the batch's titles
    news_cache: str = "auto"  # auto | hidden | none   ("vectors" = hidden + epoch_news_table on)
    # per_epoch schedule: the news vectors are constant within a local epoch (the head only
    # steps at epoch end), so encode the whole news table once per epoch and gather rows
    epoch_news_table: str = "auto"  # auto (= on when the hidden cache is) | on | off
    device_sampler: bool = True  # GPU: negative sampling + batch assembly by the HIP sampler
    # per-step GA: run the gradient all-reduce + Adam on a side stream, overlapped with the next
    # step's (parameter-free) frozen-backbone forward.  auto = GPU + all-reduce + frozen backbone
    overlap_optimizer: str = "auto"  # auto | on | off
    # per-step schedule on the device with the hidden-state cache: capture forward + backward of
    # a step in a HIP graph per (batch shape, unique-title bucket) and replay it (one launch
    # instead of ~60 host-issued kernels); the all-reduce + Adam stay eager.  auto = on there
    # unless LDP noise is on (its Philox offset advances per step on the host)
    step_graph: str = "auto"  # auto | on | off
    device: str = "auto"  # auto | cpu | cuda
    seed: int = 0

    # --- io / observability ------------------------------------------------------------
    snapshot_path: str = "snapshot.pt"
    # reference round interchange files (client.py:288 model.pt, server.py:27
    # received_model_{k}.pt), written beside snapshot_path; off by default (270 MB each)
    round_artifacts: bool = False
    metrics_path: str = ""  # JSONL; empty = metrics.jsonl beside the snapshot on rank 0
    run_name: str = "fedrec"
    wandb_project: str = "Node4"  # only used when FEDREC_WANDB=1 and wandb is importable
    verbose: bool = True

    compat: Compat = field(default_factory=Compat)

    # ------------------------------------------------------------------------------------
    def resolved_local_update(self) -> str:
        if self.local_update != "auto":
            return self.local_update
        return "per_step" if self.mode == "grad_avg" else "per_epoch"

    def quirks(self) -> Compat:
        return self.compat.resolved()

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), sort_keys=True)

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "FedRecConfig":
        cfg = FedRecConfig()
        for k, v in d.items():
            _set_dotted(cfg, k, v, flat=False)
        return cfg

    def apply_overrides(self, args: List[str]) -> List[str]:
        """Consume ``--key=value`` items; return the arguments that were not overrides."""
        rest, kv = [], []
        for a in args:
            if a.startswith("--") and "=" in a:
                k, v = a[2:].split("=", 1)
                kv.append((k.replace("-", "_"), v))
            else:
                rest.append(a)
        # --backbone.name=X selects the whole preset first; the other backbone.* overrides
        # (frozen, dropout, ...) then apply on top of it, in any argument order
        for k, v in kv:
            if k == "backbone.name":
                self.backbone = BackboneConfig.preset(v)
        for k, v in kv:
            if k != "backbone.name":
                _set_dotted(self, k, v, flat=True)
        return rest


def _coerce(old: Any, v: Any) -> Any:
    if not isinstance(v, str):
        return v
    if isinstance(old, bool):
        return v.lower() in ("1", "true", "yes", "on")
    if isinstance(old, int) and not isinstance(old, bool):
        return int(float(v))
    if isinstance(old, float):
        return float(v)
    if old is None:
        try:
            return float(v)
        except ValueError:
            return v
    return v


def _set_dotted(obj: Any, key: str, value: Any, flat: bool) -> None:
    parts = key.split(".")
    for p in parts[:-1]:
        if not hasattr(obj, p):
            raise KeyError(f"unknown config section {p!r} in {key!r}")
        obj = getattr(obj, p)
    last = parts[-1]
    if not hasattr(obj, last):
        raise KeyError(f"unknown config key {key!r}")
    old = getattr(obj, last)
    if dataclasses.is_dataclass(old) and isinstance(value, dict):
        for k, v in value.items():
            _set_dotted(old, k, v, flat=False)
        return
    setattr(obj, last, _coerce(old, value))
