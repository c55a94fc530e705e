"""The local training engine of one federated client (one process, one GPU).

Replaces the reference's ``train_on_step`` / ``UserModel.forward/collect/update`` hot path
(``client.py:61-101``, ``model.py:41-129``) with a device-resident design:

* the client's token table ``bert_news_index`` ``[N, 2, T]`` lives in HBM, and so (frozen
  backbone, ``news_cache``) do the backbone's last hidden states of every title
  (:mod:`.news_cache`): DistilBERT runs once per title per training run instead of once per
  occurrence per step (``model.py:41-61``) and again in the replay (``model.py:83-87``);
* each step de-duplicates the batch's news ids on the device (the reference re-encodes
  every occurrence: only 39 of 324 titles were unique in E8), runs the trainable head on
  the unique titles' cached hidden states, gathers rows for candidates/history, and
  scatters the per-occurrence gradients back with a deterministic segment sum
  (``client.py:26-48``) -- LDP clip + noise fused;
* no host round trip for vectors or gradients (K08, K15 removed).

Two update schedules (Q3):

``per_step`` (grad_avg / BASELINE config 2)
    forward + backward through the head for the batch's unique news, gradient all-reduce,
    one fused Adam step -- a synchronous data-parallel step.
``per_epoch`` (fedavg_star / param_avg; reference semantics)
    news vectors are fixed within a local epoch (computed in eval mode, ``model.py:42``);
    per-news gradients accumulate in an HBM table ``G [N, 400]``; at epoch end the head
    VJP replays ``G`` over the touched news (``model.py:72-90``) and both encoders take one
    Adam step (``model.py:66-70``).  ``epoch_news_table`` precomputes the whole news
    table once per epoch (exact: the head is constant within the epoch).
"""
from __future__ import annotations

import collections
import contextlib
import math
import time
from typing import Callable, Dict, NamedTuple, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..config import FedRecConfig
from ..data.sampler import DeviceSampler, HostSampler, validation_batches
from ..data.shard import Shard
from ..eval.metrics import batch_metrics
from ..models.fedrec_model import FedRecModel
from ..ops import functional as OF
from ..ops import native
from ..parallel.collcheck import CHECK
from ..utils import obs
from .news_cache import HiddenCache


def _adjacent_ids(c: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """``[cand | his]`` flattened: a view when the device sampler wrote them side by side in one
    buffer (no concatenating copy launch), else a cat."""
    if (c.is_contiguous() and h.is_contiguous() and c.dtype == h.dtype and c.device == h.device
            and c.untyped_storage().data_ptr() == h.untyped_storage().data_ptr()
            and h.storage_offset() == c.storage_offset() + c.numel()):
        return torch.empty(0, dtype=c.dtype, device=c.device).set_(c.untyped_storage(), c.storage_offset(),
                                                                   (c.numel() + h.numel(),), (1,))
    return torch.cat([c.reshape(-1), h.reshape(-1)])


class Prepared(NamedTuple):
    """A sampled batch with its dedup done ahead of time (``LocalEngine.prepare``)."""

    cand: torch.Tensor
    his: torch.Tensor
    dedup: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]]
    ready: Optional[torch.cuda.Event]
    padded: bool = False  # dedup's unique list padded with rows no occurrence maps to (step graphs)
    nreal: Optional[torch.Tensor] = None  # device int32 [1]: the real titles of a padded list
    held: bool = False  # lifetime kept by LocalEngine._retire (no per-tensor record_stream)


# "thread_local": only this thread's unsafe calls are refused during a capture -- the RCCL
# process group's watchdog thread keeps polling its work events (a multi-client run captures
# its step graphs while collectives of other steps are tracked); "global" would turn those polls
# into capture failures
_CAPTURE_MODE = "thread_local"


# N > 1: the text head's and its fc's weight gradients are written into the flat gradient buffer
# by their backward launches (ops.functional.grads_into) instead of fresh tensors that the end of
# the backward copies there; False only in the test that compares the two
INPLACE_HEAD_GRADS = True


class _StepGraph:
    """Static inputs + the captured graph of one (batch shape, unique-title bucket)."""

    def __init__(self, eng: "LocalEngine", pre: Prepared, ucap: int, with_adam: bool = False):
        uniq, inv, perm, ptr = pre.dedup
        self.adam = with_adam
        self.eng = eng
        dev = eng.device
        self.cand = torch.zeros_like(pre.cand)
        self.his = torch.zeros_like(pre.his)
        self.uniq = torch.zeros(ucap, dtype=uniq.dtype, device=dev)
        self.inv = torch.zeros_like(inv)
        self.perm = torch.zeros_like(perm)
        self.ptr = torch.zeros(ucap + 1, dtype=ptr.dtype, device=dev)
        # the real title count on the device: the text-head kernels skip the padded titles
        # (their rows carry no gradient; outputs exact zeros) -- ~5 % of the head's work at B = 64
        self.nreal = torch.zeros(1, dtype=torch.int32, device=dev)
        self._none = torch.empty(0, dtype=torch.int32, device=dev)
        # the step's weight casts + counter bumps ride in each replay's input launch (load):
        # the graph reads the compute copies from persistent buffers, no cast launch of its own
        self.precast = eng.fused_user and eng.fused_head
        self.load(pre, int(uniq.numel()), cast=False)
        static = Prepared(self.cand, self.his, (self.uniq, self.inv, self.perm, self.ptr), None, True,
                          self.nreal)
        main = torch.cuda.current_stream(dev)
        eng.sync_params()
        # two graphs: (1) the parameter-free gather of the unique titles' cached hidden states,
        # replayed BEFORE the step waits for the previous optimizer step, so the gradient
        # all-reduce + Adam on the side stream overlap it; (2) the rest of the forward + backward
        eng.hcache.ensure()
        side = torch.cuda.Stream(dev)
        self.hid_graph = None
        self.early = False  # the captured step issues the user slice's all-reduce early (N > 1)
        # (on with a gradient all-reduce only: at one client there is only Adam (7 us) to hide,
        # and the extra replay measured neutral: 66.86k vs 67.15k imp/s, r2_bench_batch6.jsonl)
        # (the fused text head reads the cache by index inside its GEMM: nothing to gather ahead)
        if not eng.fused_head and eng.grad_allreduce is not None:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                for _ in range(2):
                    self.hid = eng.hcache.rows(self.uniq)
            main.wait_stream(side)
            self.hid_graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.hid_graph, capture_error_mode=_CAPTURE_MODE):
                self.hid = eng.hcache.rows(self.uniq)
            eng._pre_hid = self.hid
        # warm up on a side stream (autograd / allocator state), then capture on it
        try:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                for _ in range(2):
                    eng.forward_backward(self.cand, self.his, static)
            main.wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            # a private memory pool per graph (~250 MB of step activations at B = 64): sharing
            # the first graph's pool (graph.pool()) trips an allocator assert in this torch build
            # when eager steps of other engines run between the captures
            # in-graph Adam: the step's cast launch (its first kernel) advances the device step count
            eng._adam_bump = eng._adam_step_dev if with_adam else None
            # the in-graph Adam gathers the step's gradients from where autograd left them and
            # writes them into the flat buffer itself: no separate copy launch (6 us per step) --
            # unless a gradient all-reduce sits between them (N > 1): it needs the flat buffer
            ar = eng.grad_allreduce if with_adam else None
            eng._adam_gathers = with_adam and ar is None
            eng._precast = eng.step_cast_bufs() if self.precast else None
            # N > 1 with the IPC all-reduce: the user encoder's slice is reduced early, inside the
            # backward (a side-stream branch of the graph); only while capturing -- the warm-ups
            # above run on one rank only when its bucket is new, and must not issue collectives
            early = (ar is not None and eng._ar_side is not None and getattr(ar, "split", None))
            hook = OF.after_user_wgrads(eng._early_user_reduce) if early else contextlib.nullcontext()
            eng._early_issued = False
            with torch.cuda.graph(self.graph, capture_error_mode=_CAPTURE_MODE):
                with hook:
                    self.loss = eng.forward_backward(self.cand, self.his, static)
                if with_adam:  # the step in one graph: backward, [all-reduce,] Adam
                    if eng._early_issued:
                        scale = ar.finish_early(eng.flat.grad, eng._ar_side)
                    else:
                        scale = ar(eng.flat.grad) if ar is not None else 1.0
                    eng._adam_dev(self.loss, scale)
            self.early = eng._early_issued
        finally:
            eng._early_issued = False
            eng._pre_hid = None
            eng._adam_bump = None
            eng._adam_gathers = False
            eng._grad_srcs = None
            eng._precast = None

    def load(self, pre: Prepared, U: int, cast: bool = True) -> None:
        """The batch into the static inputs: one launch; the unique list is padded with news 0
        and the segment pointers with R (padded segments are empty).  ``cast`` (a replay of a
        graph captured with persistent compute copies): the same launch casts the step's weights
        into them and advances the step counters (csrc/adam.hip multi_cast, copy segments) --
        the separate in-graph cast launch was 5 us per step."""
        uniq, inv, perm, ptr = pre.dedup
        src = [pre.cand.contiguous(), pre.his.contiguous(), uniq, inv, perm, ptr, self._none]
        dst = [self.cand, self.his, self.uniq, self.inv, self.perm, self.ptr, self.nreal]
        fill = [0, 0, 0, 0, 0, int(inv.numel()), U]
        lib = native.require_for(self.cand)
        if cast and self.precast:
            eng = self.eng
            csrc, cdst = eng.step_cast_lists()
            lib.copy_cast(src, dst, fill, csrc, cdst, eng._rng_step, eng._adam_step_dev if self.adam else None)
        else:
            lib.multi_copy(src, dst, fill)


class LocalEngine:
    def __init__(self, cfg: FedRecConfig, model: FedRecModel, shard: Shard, device: torch.device,
                 rank: int = 0, grad_allreduce: Optional[Callable[[torch.Tensor], float]] = None):
        if device.type == "cuda" and cfg.precision != "bf16":
            raise ValueError(f"precision={cfg.precision!r} on the device: the HIP kernels compute in bf16 "
                             "(fp32 is the host/oracle path; there is no eager fallback on the device)")
        self.cfg = cfg
        self.q = cfg.quirks()
        self.model = model
        self.shard = shard
        self.device = device
        self.rank = rank
        self.flat = model.flat if model.flat is not None else model.build_flat()
        self.tokens = torch.as_tensor(shard.news_index, dtype=torch.int32).to(device)  # HBM resident
        self.N = shard.num_news
        if device.type == "cuda" and cfg.device_sampler:
            self.sampler = DeviceSampler(shard.train, cfg.batch_size, device, cfg.npratio, cfg.max_his_len,
                                         truncate=not self.q.no_history_truncation, seed=cfg.seed, rank=rank)
        else:
            self.sampler = HostSampler(shard.train, cfg.batch_size, cfg.npratio, cfg.max_his_len,
                                       truncate=not self.q.no_history_truncation, seed=cfg.seed, rank=rank)
        # grad_allreduce(flat_grad) -> scale to apply (1/W); None = local only
        self.grad_allreduce = grad_allreduce
        # the user encoder's parameters are the flat buffer's tail (registration order): at N > 1
        # the IPC all-reduce sends that slice in its own call, early (see _early_user_reduce)
        self._user_first = self._user_slice_start(model)
        self._ar_side = None
        self._early_issued = False
        if (grad_allreduce is not None and getattr(grad_allreduce, "kind", "") == "ipc"
                and hasattr(grad_allreduce, "split") and self._user_first is not None):
            grad_allreduce.split = self.flat.offsets[self._user_first]
            self._ar_side = torch.cuda.Stream(device)
        # or a BucketReducer (large trainable sets: the unfrozen backbone): buckets reduced
        # during the backward as their gradients land (set_reducer)
        self.reducer = None
        self.sigma: Optional[float] = None  # LDP noise multiplier (set by the client driver)
        self.noise_offset = 0
        self.epoch = 0
        self.G: Optional[torch.Tensor] = None
        self.touched: Optional[torch.Tensor] = None
        self.news_table: Optional[torch.Tensor] = None
        # train-mode dropout masks of the backbone (unfrozen training, Q4 replay): Philox key per client
        model.text_encoder.DistillBert.drop_seed = (int(cfg.seed) << 20) + 7919 * int(rank) + 1
        # device user side as one fused autograd Function (ops.functional.UserStepFn): our GEMMs
        # and kernels end to end; the user-input dropout mask is Philox keyed by (seed, step),
        # the step being a device counter so HIP-graph replays draw fresh masks
        ue = model.user_encoder
        self.fused_user = (device.type == "cuda"
                           and ue.multihead_attention.n_heads * ue.multihead_attention.d_k == cfg.news_dim)
        self.user_drop_seed = (int(cfg.seed) << 20) + 7919 * int(rank) + 2
        ue.drop_seed = self.user_drop_seed  # the module-level device path (user_encoder_device) too
        # LDP noise: its own Philox key per client (disjoint from the dropout keys above)
        self.ldp_seed = (int(cfg.seed) << 20) + 7919 * int(rank) + 3
        self._rng_step = torch.zeros(1, dtype=torch.int64, device=device)
        self._adam_bump = None  # set while capturing a step graph with Adam in it (see _StepGraph)
        self._adam_gathers = False  # ... and then Adam gathers the gradients (no end_backward copy)
        self._precast = None  # set while capturing: the step's compute copies, filled before each replay
        self._cast_bufs = None
        self._cast_lists = None
        self._grad_srcs = None
        self._inflight = collections.deque()  # (held batch, end event or None), see _retire
        self._held_n = 0
        # hidden states of the step's unique titles gathered ahead (the step graph's first part)
        self._pre_hid: Optional[torch.Tensor] = None
        self._one: Optional[torch.Tensor] = None  # seed gradient of the loss (see forward_backward)
        self.hcache = self._make_hidden_cache()
        self.catalog = None  # (CatalogPlan, data group): cooperative cache builds (set_catalog)
        self.catalog_refused: Optional[str] = None  # why parallel.catalog.attach fell back to local builds
        # host-batch validation: encode the whole news table first (auto: when the batches would
        # touch more titles than it has) | never | always -- the tests pin both forms
        self.valid_table = "auto"
        self._catalog_ctrl = None
        self.epoch_table = (cfg.epoch_news_table == "on" or cfg.news_cache == "vectors"
                            or (cfg.epoch_news_table == "auto" and self.hcache is not None))
        self.replay_chunk = 4096 if self.hcache is not None else 1024
        # HIP graphs of the per-step forward + backward (see _graph_step)
        sg = cfg.step_graph
        self.step_graphs = device.type == "cuda" and self.hcache is not None and (
            sg == "on" or (sg == "auto" and (self.fused_user or not cfg.dp.enabled)))
        self._graphs: Dict[tuple, "_StepGraph"] = {}
        self.last_stats: Dict[str, float] = {}
        # step counters (tests / bench): graph replays, replays that ran the all-reduce + Adam
        # inside the graph, and optimizer steps issued eagerly from the host
        self.counts = {"replays": 0, "replays_with_optimizer": 0, "eager_optimizer_steps": 0, "eager_steps": 0,
                       "captures": 0, "early_reduces": 0}
        self.inplace_grads = 0
        self.host_wait_s = 0.0  # host time blocked on the run-ahead bound (_retire): the DEVICE is the limit
        # optimizer overlap (per-step schedule): grads all-reduced + Adam on a side stream while
        # the next step samples, dedups and runs the frozen backbone, none of which reads the
        # trainable parameters; everything that does calls sync_params() first
        ov = cfg.overlap_optimizer
        self.overlap = device.type == "cuda" and cfg.backbone.frozen and (
            ov == "on" or (ov == "auto" and grad_allreduce is not None))
        self._side = torch.cuda.Stream(device) if self.overlap else None
        self._params_ready: Optional[torch.cuda.Event] = None
        # batch lookahead (GPU): the next batch is sampled and de-duplicated on its own stream
        # while the current step runs, so the dedup's host read of the unique count (the
        # backbone's M) no longer drains the GPU at every step start
        self._prep = torch.cuda.Stream(device) if device.type == "cuda" else None

    def _grad_slots(self) -> Dict[int, torch.Tensor]:
        """id(parameter) -> its slot of the flat gradient buffer (a view of the parameter's shape)."""
        if getattr(self, "_slots", None) is None:
            fl = self.flat
            self._slots = {id(p): fl.grad[off:off + p.numel()].view_as(p) for p, off in zip(fl.params, fl.offsets)}
        return self._slots

    def _user_slice_start(self, model) -> Optional[int]:
        """Index of the first user-encoder parameter in the flat buffer when the user encoder's
        parameters form its tail (contiguous, after every other one), else None."""
        ids = {id(p) for p in model.user_encoder.parameters() if p.requires_grad}
        flags = [id(p) in ids for p in self.flat.params]
        if not any(flags):
            return None
        i0 = flags.index(True)
        return i0 if i0 > 0 and all(flags[i0:]) else None

    def _early_user_reduce(self) -> None:
        """Called inside the captured backward once the user encoder's weight gradients are final
        (ops.functional.after_user_wgrads: after the text fc's backward launch that computes
        them): their slots of the flat gradient get them (one copy launch) and the IPC all-reduce
        of that slice starts on a side stream -- beside the text head's pool backward and weight
        gradient, ~130 us of the step -- as DDP's first bucket fires inside ``loss.backward()``
        (``Gradient_Averaging_main.py:119``).  The head slice follows after the backward
        (grad_allreduce.finish_early)."""
        fl = self.flat
        src, dst = [], []
        for p, off in zip(fl.params[self._user_first:], fl.offsets[self._user_first:]):
            view = fl.grad[off:off + p.numel()].view_as(p)
            g = p.grad
            if g is None:
                view.zero_()
            elif g.data_ptr() != view.data_ptr():
                src.append(g if g.is_contiguous() and g.dtype == torch.float32 else g.float().contiguous())
                dst.append(view)
            p.grad = view  # end_backward leaves these slots alone
        if src and not native.require_for(fl.grad).multi_cast(src, dst):
            torch._foreach_copy_(dst, src)
        self.grad_allreduce.early(fl.grad, self._ar_side)
        self._early_issued = True

    def set_reducer(self, reducer) -> None:
        """Use a backward-overlapped bucket reducer (``parallel.reducer``) for the gradients."""
        self.reducer = reducer

    def check_data_plane(self) -> None:
        """Raise if a gradient all-reduce failed silently on the device (the IPC all-reduce
        records a peer timeout in a status word and poisons that call's output); one device
        read, at every epoch end."""
        for obj in (self.grad_allreduce, self.reducer):
            chk = getattr(obj, "check", None)
            if chk is not None:
                chk()

    def state(self) -> Dict[str, int]:
        """Counters that key the engine's randomness (checkpointed with the snapshot)."""
        return {"noise_offset": self.noise_offset, "epoch": self.epoch,
                "drop_calls": self.model.text_encoder.DistillBert._drop_calls,
                "user_drop_calls": int(getattr(self.model.user_encoder, "drop_calls", 0)),
                "rng_step": int(self._rng_step.item())}

    def load_state(self, st: Dict[str, int]) -> None:
        self.noise_offset = int(st.get("noise_offset", self.noise_offset))
        self._rng_step.fill_(int(st.get("rng_step", 0)))  # user-dropout / LDP-noise step counter
        self.epoch = int(st.get("epoch", self.epoch))
        self.model.text_encoder.DistillBert._drop_calls = int(st.get("drop_calls", 0))
        self.model.user_encoder.drop_calls = int(st.get("user_drop_calls", 0))

    def _make_hidden_cache(self) -> Optional[HiddenCache]:
        """The HBM hidden-state cache when the config asks for it and it fits."""
        mode = self.cfg.news_cache
        if mode == "none" or not self.cfg.backbone.frozen:
            return None
        te = self.model.text_encoder
        if mode in ("auto", "vectors"):
            if self.device.type != "cuda":
                return None
            need = HiddenCache.nbytes_for(self.N, self.tokens.shape[2], self.cfg.backbone.dim, te.compute_dtype)
            free, _ = torch.cuda.mem_get_info(self.device)
            if need > free // 4:
                obs.log(f"[rank {self.rank}] hidden-state cache off: {need / 2**30:.1f} GiB > 1/4 of "
                        f"{free / 2**30:.1f} GiB free")
                return None
        elif mode != "hidden":
            raise ValueError(f"news_cache={mode!r}: expected auto | hidden | none | vectors")
        return HiddenCache(te, self.tokens)

    def set_catalog(self, plan, data_group, ctrl_group=None) -> None:
        """Cooperative cache builds (:mod:`..parallel.catalog`): :meth:`build_cache` encodes this
        client's 1/W share of the catalog and all-gathers the rest over ``data_group``.  Every
        client of the group must then call :meth:`build_cache` at the same points; the lazy
        rebuild of a stale cache inside a step (:meth:`HiddenCache.ensure`) stays a local build."""
        self.catalog = (plan, data_group) if plan is not None else None
        self._catalog_ctrl = ctrl_group

    def build_cache(self) -> Optional[float]:
        """(Re)build the hidden-state cache now; returns its build time in seconds (None: no cache).
        With a catalog plan (:meth:`set_catalog`) this is a collective over the clients."""
        if self.hcache is None:
            return None
        self.sync_params()
        if self.catalog is not None:
            return self.hcache.build(*self.catalog)
        return self.hcache.build()

    def ensure_cache(self) -> None:
        """Collective point of the round drivers: rebuild a stale cache now (cooperatively when a
        catalog plan is set) instead of lazily inside the first step."""
        if self.hcache is None:
            return
        stale = not self.hcache.fresh()
        if self.catalog is not None and self._catalog_ctrl is not None:
            # the clients agree first (one gloo MAX): any stale cache -> every client rebuilds, so
            # the cooperative gather never waits for a client that thought its table was fresh
            import torch.distributed as dist

            t = torch.tensor([1 if stale else 0], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self._catalog_ctrl)
            stale = bool(t.item())
        if stale:
            self.build_cache()

    # -------------------------------------------------------------------------------
    @property
    def score_act(self) -> str:
        return self.cfg.score_act

    def _ldp(self):
        """(clip, noise std) for the per-occurrence news gradients (client.py:87-89)."""
        if not self.cfg.dp.enabled or not self.sigma:
            return 0.0, 0.0
        if self.q.ldp_no_clip:  # Q10: no clipping, std = sigma
            return 0.0, float(self.sigma)
        return float(self.cfg.dp.clip), float(self.sigma * self.cfg.dp.clip)

    def to_device(self, a) -> torch.Tensor:
        if isinstance(a, torch.Tensor):
            return a.to(self.device, non_blocking=True)
        t = torch.from_numpy(np.ascontiguousarray(a))
        if self.device.type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t

    def step_cast_bufs(self):
        """Persistent compute copies of the step's weights (shared by every step graph)."""
        if self._cast_bufs is None:
            self._cast_bufs = OF.step_cast_buffers(self.model.text_encoder, self.model.user_encoder)
        return self._cast_bufs

    def step_cast_lists(self):
        """``(sources, destinations)`` of the weight casts into :meth:`step_cast_bufs`."""
        te, ue = self.model.text_encoder, self.model.user_encoder
        # (cached: rebuilding the slices costs ~50 us of host time per step; keyed on where the
        # weights live, so a re-bound parameter is never cast from its old storage)
        key = (te.fc.weight.data_ptr(), te.additive_attention.att_fc1.weight.data_ptr(),
               ue.multihead_attention.W_Q.weight.data_ptr())
        if self._cast_lists is None or self._cast_lists[0] != key:
            self._cast_lists = (key, OF.step_cast_lists(te, ue, self.step_cast_bufs()))
        return self._cast_lists[1]

    def sync_params(self) -> None:
        """Make the current stream wait for a pending overlapped optimizer step."""
        if self._params_ready is not None:
            torch.cuda.current_stream(self.device).wait_event(self._params_ready)
            self._params_ready = None

    def _hidden(self, ids: torch.Tensor):
        """Backbone hidden states ``[n, T, D]`` of titles ``ids`` and their token masks (the
        mask only when the head uses it).  From the HBM cache when it is on; otherwise the
        frozen / unfrozen backbone runs on the titles."""
        if self.hcache is not None:
            hid = self._pre_hid if self._pre_hid is not None else self.hcache.rows(ids)
            mask = self.tokens.index_select(0, ids.long())[:, 1, :] if self.cfg.mask_padding else None
            return hid, mask
        text = self.tokens.index_select(0, ids.long())
        return self.model.text_encoder.hidden(text), text[:, 1, :]

    @property
    def fused_head(self) -> bool:
        """Text head on the fused kernels straight over the hidden-state cache (by index)."""
        return self.hcache is not None and self.model.text_encoder.fused_head_ok(self.tokens.shape[2])

    def _cache_ids(self, ids: torch.Tensor) -> torch.Tensor:
        return ids if ids.dtype == torch.int32 else ids.to(torch.int32)

    def news_vectors(self, uniq: torch.Tensor, grad: bool, nreal: Optional[torch.Tensor] = None,
                     w1b: Optional[torch.Tensor] = None, fcb: Optional[torch.Tensor] = None) -> torch.Tensor:
        """News vectors of titles ``uniq``; ``nreal`` (device int32 [1], fused head only): rows
        past it are padding of a step graph's unique list and come out as the fc bias."""
        te = self.model.text_encoder
        if not grad and self.news_table is not None:
            return self.news_table.index_select(0, uniq.long())
        if self.fused_head:
            table = self.hcache.flat()
            self.sync_params()
            if grad:
                return te.head_rows(table, self._cache_ids(uniq), self.tokens.shape[2], self.tokens, nreal, w1b, fcb)
            with torch.no_grad():
                return te.head_rows(table, self._cache_ids(uniq), self.tokens.shape[2], self.tokens)
        hid, mask = self._hidden(uniq)  # parameter-free: overlaps the previous step's all-reduce + Adam
        self.sync_params()
        if grad:
            return te.head(hid, mask)
        with torch.no_grad():
            return te.head(hid, mask)

    # -------------------------------------------------------------------------------
    @property
    def DEDUP_SYNC_MAX(self) -> int:
        """Ids up to which the native dedup is one kernel chain ending in its unique-count read
        (so no event is needed for the main stream); the extension's own constant, read once."""
        v = getattr(LocalEngine, "_dedup_sync_max", None)
        if v is None:
            v = int(native.lib().dedup_sync_max()) if self.device.type == "cuda" else 0
            LocalEngine._dedup_sync_max = v
        return v

    def prepare(self, batch_fn: Callable[[], Tuple], held: bool = False) -> Prepared:
        """Sample a batch (``batch_fn() -> (cand, his)``) and de-duplicate its news ids.  On the
        GPU both run on the lookahead stream: the only host wait (the unique count) waits for
        that stream alone, so a step's dedup overlaps the previous step's kernels.
        ``batch_fn`` must produce its tensors on the lookahead stream (the device sampler does,
        via :meth:`_next_prepared`) or return host arrays / tensors already complete: the
        lookahead stream does not wait for other streams."""
        if self._prep is None:
            c, h = batch_fn()
            return Prepared(self.to_device(c), self.to_device(h), None, None)
        main = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self._prep):
            c, h = batch_fn()
            c, h = self.to_device(c), self.to_device(h)
            ids = _adjacent_ids(c, h)
            dd = ops.dedup(ids, self.N)
            ev = None
            if ids.numel() > self.DEDUP_SYNC_MAX:  # the sort path queues work after its count read
                ev = torch.cuda.Event()
                ev.record(self._prep)
        if not held:  # (held: the training loop keeps the batch alive -- see _retire)
            for t in (c, h, *dd):
                t.record_stream(main)
        # otherwise no event for the main stream to wait on: the dedup's unique count is a host
        # read on the lookahead stream, the last work queued there for this batch, so when it
        # returns every lookahead kernel of the batch has completed (kernel completion publishes
        # its writes at agent scope).  A per-step hipStreamWaitEvent measured ~33 us of device
        # idle between steps (profiles/r4_graph_gap.json).
        return Prepared(c, h, tuple(dd), ev, held=held)

    def _forward_rows(self, cand: torch.Tensor, his: torch.Tensor, grad_news: bool, pre: Optional[Prepared] = None):
        B, C = cand.shape
        H = his.shape[1]
        if pre is not None and pre.dedup is not None:
            if pre.ready is not None:
                torch.cuda.current_stream(self.device).wait_event(pre.ready)
            uniq, inv, perm, ptr = pre.dedup
        else:
            ids = _adjacent_ids(cand, his)
            uniq, inv, perm, ptr = ops.dedup(ids, self.N)
        with obs.range("news_encode"):
            v = self.news_vectors(uniq, grad=grad_news)
        if not grad_news:
            v = v.detach().requires_grad_(True)
        clip, std = self._ldp()
        padded = pre is not None and pre.padded
        rows = OF.news_gather(v, inv, perm, ptr, clip, std, self.ldp_seed, (1 << 40) + self.noise_offset, padded)
        self.noise_offset += 1
        cand_v = rows[: B * C].view(B, C, -1)
        his_v = rows[B * C:].view(B, H, -1)
        return uniq, v, cand_v, his_v

    def _user_loss(self, v: torch.Tensor, dd, B: int, C: int, H: int, padded: bool, train: bool,
                   his: Optional[torch.Tensor] = None, casts=None):
        """Device user side (fused): ``(loss, scores)`` from news vectors ``v`` of the unique ids.
        ``his [B, H]``: the batch's history ids, the key mask when ``mask_padding`` is on."""
        uniq, inv, perm, ptr = dd
        p = float(self.cfg.user_dropout) if train else 0.0
        clip, std = self._ldp()
        # the fused path's noise offset is the device step counter alone (_rng_step, advanced once per
        # step inside the step graph too): the host part is a constant, so eager and replayed steps
        # never reuse an offset; the non-fused path (news_gather) keeps the host counter, offset
        # past 2^40 so the two streams cannot meet
        ldp = (clip, std, self.ldp_seed, 0)
        if train:
            self.noise_offset += 1
        keep = his if (self.cfg.mask_padding and his is not None) else None
        return OF.user_step(v, inv, perm, ptr, self.model.user_encoder, B, C, H, self.score_act,
                            (p, self.user_drop_seed, 0), self._rng_step, ldp, padded, keep, self._seed_one(), casts)

    def _seed_one(self) -> torch.Tensor:
        """The persistent ones tensor every fused backward is seeded with (no fill launch per
        step; the captured graph reads it in place, and UserStepFn skips the scale by it)."""
        if self._one is None or self._one.device != self.device:
            self._one = torch.ones((), device=self.device, dtype=torch.float32)
        return self._one

    def _dedup(self, cand, his, pre):
        if pre is not None and pre.dedup is not None:
            if pre.ready is not None:
                torch.cuda.current_stream(self.device).wait_event(pre.ready)
            return pre.dedup
        return tuple(ops.dedup(_adjacent_ids(cand, his), self.N))

    def forward_backward(self, cand: torch.Tensor, his: torch.Tensor, pre: Optional[Prepared] = None) -> torch.Tensor:
        """Loss of one batch with every trainable gradient left in ``flat.grad``."""
        self.model.train()
        if self.epoch_table or not self.cfg.backbone.frozen:
            self.sync_params()
        self.flat.begin_backward()
        if self.reducer is not None:
            self.reducer.begin()
        if self.fused_user:
            dd = self._dedup(cand, his, pre)
            casts = None
            if self.fused_head:  # every compute copy of the step's weights in one cast launch,
                self.sync_params()  # which also advances the dropout / noise step counter this step reads
                if self._precast is not None:  # a step graph: its replay's input launch casts them
                    casts = self._precast
                else:
                    casts = OF.step_weight_casts(self.model.text_encoder, self.model.user_encoder,
                                                 bump=self._rng_step, bump2=self._adam_bump)
            # N > 1: the text head's and fc's weight gradients straight into the flat buffer (the
            # all-reduce reads them there; no end-of-backward copy of six fresh tensors)
            into = (OF.grads_into(self._grad_slots()) if INPLACE_HEAD_GRADS and self.grad_allreduce is not None
                    and self.reducer is None and not self._adam_gathers else contextlib.nullcontext())
            with into:
                with obs.range("news_encode"):
                    v = self.news_vectors(dd[0], grad=True, nreal=pre.nreal if pre is not None else None,
                                          w1b=casts[0] if casts is not None else None,
                                          fcb=casts[2] if casts is not None else None)
                with obs.range("user_step"):
                    loss, _ = self._user_loss(v, dd, cand.shape[0], cand.shape[1], his.shape[1],
                                              pre is not None and pre.padded, True, his,
                                              casts=casts[1] if casts is not None else None)
                # weight gradients beside the rest of the backward (fresh .grad: begin_backward
                # above; a bucket reducer's per-gradient hooks would read them before the side
                # stream ran)
                side = OF.side_wgrads() if self.reducer is None else contextlib.nullcontext()
                with obs.range("backward"), side:
                    loss.backward(self._seed_one())
            inplace = OF.take_written()
            self.inplace_grads = len(inplace)  # (tests: how many slots the last backward wrote in place)
            if casts is None:
                self._rng_step.add_(1)  # next step's dropout masks (inside a captured graph too)
            if self._adam_gathers:  # the in-graph Adam reads the fresh gradients where they are
                self._grad_srcs = self.flat.end_backward(copy=False, inplace=inplace)
            else:
                self.flat.end_backward(inplace=inplace)
            return loss.detach()
        _, _, cand_v, his_v = self._forward_rows(cand, his, grad_news=True, pre=pre)
        with obs.range("user_fwd"):
            u = self.model.user_encoder(his_v, his)
            loss, _ = OF.score_ce(cand_v, u, self.score_act)
        with obs.range("backward"):
            loss.backward()
        self.flat.end_backward()
        return loss.detach()

    def train_step(self, cand: torch.Tensor, his: torch.Tensor, pre: Optional[Prepared] = None) -> torch.Tensor:
        """``per_step`` schedule: grads -> all-reduce -> Adam.  Returns the (device) loss."""
        loss = self.forward_backward(cand, his, pre)
        self.optimizer_step(overlap=True)
        return loss

    def train_prepared(self, pre: Prepared) -> torch.Tensor:
        # LDP: the fused user step draws its noise at a device-counter offset, so it replays fresh
        # noise; the non-fused path's host offset would be frozen into the graph
        if self.step_graphs and pre.dedup is not None and not (self.cfg.dp.enabled and self.sigma
                                                               and not self.fused_user):
            # (the device step count rides in the fused step's cast launch); a capturable gradient
            # all-reduce (the device-epoch IPC one) joins them: one replay per step at N > 1 too
            ar_ok = self.grad_allreduce is None or getattr(self.grad_allreduce, "capturable", False)
            with_adam = ar_ok and self.reducer is None and self.fused_user and self.fused_head
            loss = self._graph_step(pre, with_adam)
            if loss is not None:
                if not with_adam:
                    self.optimizer_step(overlap=True)
                self._retire(pre)
                return loss
        self.counts["eager_steps"] += 1
        loss = self.train_step(pre.cand, pre.his, pre)
        self._retire(pre)
        return loss

    # ---- Adam inside the step graph (no gradient all-reduce: one client) ----------------
    LOSS_RING = 4096  # per-step losses live here until read (train_epoch folds every LOSS_RING / 2)

    def _adam_dev(self, loss: torch.Tensor, scale: float = 1.0) -> None:
        """Adam with its step count on the device (csrc/adam.hip adam_dev_kernel), capturable:
        also copies the step's loss into the loss ring.  The host mirror ``flat.step`` is
        advanced by the caller per replay."""
        c = self.cfg
        srcs, self._grad_srcs = self._grad_srcs, None
        # a device-epoch IPC all-reduce in the graph: its status word makes Adam skip the update of
        # a step whose sum timed out (poisoned), and that step's loss reads NaN
        ipc = getattr(self.grad_allreduce, "ipc", None) if self.grad_allreduce is not None else None
        skip = ipc.status_word() if ipc is not None else None
        native.require_for(loss).adam_dev(self.flat.flat, self.flat.grad, self.flat.m, self.flat.v, self._adam_step_dev,
                                          loss.reshape(1).float(), self._loss_ring, c.lr, c.adam_beta1, c.adam_beta2,
                                          c.adam_eps, float(scale), srcs,
                                          list(self.flat.offsets) if srcs is not None else None, skip)

    # ---- HIP graph of the per-step forward + backward ------------------------------------
    GRAPH_BUCKET = 128  # unique titles are padded up to a multiple of this (padded rows: id 0)
    MAX_GRAPHS = 16

    def _graph_step(self, pre: Prepared, with_adam: bool = False) -> Optional[torch.Tensor]:
        """Forward + backward of one step by replaying a captured HIP graph.

        The step's only data-dependent shape is the number U of unique titles: it is padded to
        a multiple of GRAPH_BUCKET with news id 0, whose rows no occurrence maps to -- their
        head outputs are never gathered and their per-news gradient (a segment sum over no
        occurrences) is 0, so the trainable gradient is the eager step's (up to fp32
        summation order in the split-K weight gradients).  One graph per (batch shape, bucket,
        cache build); the batch is copied into the graph's static inputs, then one replay
        runs ~60 kernels with no host in between.  ``with_adam`` (no gradient all-reduce): the
        graph ends with the device-step Adam and the loss goes to the loss ring -- no eager
        launch between two steps' graphs.  Returns None when a new graph is not allowed (the
        caller runs the step eagerly)."""
        uniq, inv, perm, ptr = pre.dedup
        U = int(uniq.numel())
        ucap = -(-U // self.GRAPH_BUCKET) * self.GRAPH_BUCKET
        # a backbone sync (sync=full, an unfrozen step) may have invalidated the cache since the
        # last replay: rebuild it BEFORE keying, so a replay never reads a stale table and a new
        # graph is filed under the build it captured
        self.sync_params()
        self.hcache.ensure()
        key = (tuple(pre.cand.shape), tuple(pre.his.shape), int(inv.numel()), ucap, with_adam, self.hcache.builds)
        g = self._graphs.get(key)
        main = torch.cuda.current_stream(self.device)
        if pre.ready is not None:
            main.wait_event(pre.ready)
        if g is None:
            if len(self._graphs) >= self.MAX_GRAPHS:
                return None
            if any(k[-1] != self.hcache.builds for k in self._graphs):  # a rebuilt cache: old graphs are stale
                self._graphs = {k: v for k, v in self._graphs.items() if k[-1] == self.hcache.builds}
            if with_adam and getattr(self, "_adam_step_dev", None) is None:  # (outside any capture)
                self._adam_step_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
                self._loss_ring = torch.zeros(self.LOSS_RING, dtype=torch.float32, device=self.device)
                self._adam_mirror = -1
            g = _StepGraph(self, pre, ucap, with_adam)
            self._graphs[key] = g
            self.counts["captures"] += 1
        if not g.precast:
            g.load(pre, U)
        if g.hid_graph is not None:
            g.hid_graph.replay()  # parameter-free: runs while the previous all-reduce + Adam finish
        self.sync_params()
        if g.adam and self._adam_mirror != self.flat.step:  # an eager step / a resume moved the host count
            self._adam_step_dev.fill_(self.flat.step)
            self._adam_mirror = self.flat.step
        if g.precast:  # after the parameters' last update: this launch casts them (and bumps the counters)
            g.load(pre, U)
        self.counts["replays"] += 1
        if g.adam:
            g.graph.replay()
            ar = self.grad_allreduce
            if ar is not None:  # the captured all-reduce ran in this replay (the eager path's records)
                sp = getattr(ar, "split", None)
                if sp:
                    CHECK.record("all_reduce", self.flat.grad[sp:], "grad-ipc-user")
                    CHECK.record("all_reduce", self.flat.grad[:sp], "grad-ipc-head")
                else:
                    CHECK.record("all_reduce", self.flat.grad,
                                 "grad-ipc" if getattr(ar, "kind", "") == "ipc" else "grad")
                if g.early:
                    self.counts["early_reduces"] += 1
            self.counts["replays_with_optimizer"] += 1
            self.flat.step += 1
            self._adam_mirror += 1
            return self._loss_ring[(self.flat.step - 1) % self.LOSS_RING]
        g.graph.replay()
        return g.loss.clone()

    def optimizer_step(self, extra_scale: float = 1.0, overlap: bool = False) -> None:
        """All-reduce the flat gradient (if any) and take one fused Adam step.  ``overlap``
        (per-step schedule only): enqueue both on the side stream and return at once; the
        next reader of the parameters waits in :meth:`sync_params`."""
        if overlap and self.overlap:
            main = torch.cuda.current_stream(self.device)
            self._side.wait_stream(main)  # the gradients of this step are complete
            with torch.cuda.stream(self._side):
                self._optimizer_step(extra_scale)
                ev = torch.cuda.Event()
                ev.record(self._side)
            self._params_ready = ev
            return
        self.sync_params()
        self._optimizer_step(extra_scale)

    def _optimizer_step(self, extra_scale: float) -> None:
        self.counts["eager_optimizer_steps"] += 1
        scale = extra_scale
        if self.reducer is not None:
            with obs.range("allreduce_wait"):
                scale *= self.reducer.finish()
        elif self.grad_allreduce is not None:
            with obs.range("allreduce"):
                scale *= self.grad_allreduce(self.flat.grad)
        self.flat.step += 1
        c = self.cfg
        with obs.range("adam"):
            ops.adam_flat(self.flat.flat, self.flat.grad, self.flat.m, self.flat.v, self.flat.step,
                          c.lr, c.adam_beta1, c.adam_beta2, c.adam_eps, scale)
        if not self.cfg.backbone.frozen:
            self.model.text_encoder.DistillBert.invalidate()

    # -------------------------------------------------------------------------------
    def _begin_epoch_accumulate(self) -> None:
        self.sync_params()
        D = self.cfg.news_dim
        self.G = torch.zeros(self.N, D, dtype=torch.float32, device=self.device)
        self.touched = torch.zeros(self.N, dtype=torch.bool, device=self.device)
        self.flat.zero_grad()
        if self.epoch_table:
            self.news_table = self.encode_all(grad=False)

    @torch.no_grad()
    def encode_all(self, grad: bool = False, chunk: int = 2048) -> torch.Tensor:
        """Every title's news vector ``[N, 400]`` fp32 (eval mode).  Over the hidden-state cache
        the fused head runs the whole table in one call (three launches: score, pool, fc -- the
        title index is the cache row); otherwise in chunks of ``chunk`` titles."""
        self.sync_params()
        self.model.eval()
        if self.fused_head:
            return self.model.text_encoder.head_rows(self.hcache.flat(), None, self.tokens.shape[2], self.tokens).float()
        out = torch.empty(self.N, self.cfg.news_dim, dtype=torch.float32, device=self.device)
        for s in range(0, self.N, chunk):
            ids = torch.arange(s, min(s + chunk, self.N), device=self.device, dtype=torch.int32)
            if self.fused_head:
                out[s:s + len(ids)] = self.model.text_encoder.head_rows(self.hcache.flat(), ids, self.tokens.shape[2],
                                                                        self.tokens)
                continue
            hid, mask = self._hidden(ids)
            out[s:s + len(ids)] = self.model.text_encoder.head(hid, mask).float()
        return out

    def accumulate_step(self, cand: torch.Tensor, his: torch.Tensor, pre: Optional[Prepared] = None) -> torch.Tensor:
        """``per_epoch`` schedule: user grads + per-news gradient table, no optimizer step."""
        self.model.train()
        if self.q.grad_double_last_batch:
            self.flat.grad.zero_()  # Q2: optimizer.zero_grad() each batch (client.py:75)
        self.model.text_encoder.eval()  # gen_news_vecs runs the text encoder in eval (model.py:42)
        if self.fused_user:
            dd = self._dedup(cand, his, pre)
            v = self.news_vectors(dd[0], grad=False).detach().requires_grad_(True)
            loss, _ = self._user_loss(v, dd, cand.shape[0], cand.shape[1], his.shape[1], False, True, his)
            loss.backward(self._seed_one())
            self._rng_step.add_(1)
            self.G.index_add_(0, dd[0].long(), v.grad)
            self.touched[dd[0].long()] = True
            return loss.detach()
        uniq, v, cand_v, his_v = self._forward_rows(cand, his, grad_news=False, pre=pre)
        u = self.model.user_encoder(his_v, his)
        loss, _ = OF.score_ce(cand_v, u, self.score_act)
        loss.backward()
        self.G.index_add_(0, uniq.long(), v.grad)
        self.touched[uniq.long()] = True
        return loss.detach()

    def end_epoch_update(self, n_steps: int) -> None:
        """Replay the per-news gradients through the head, then one Adam step."""
        if n_steps == 0:
            return
        self.sync_params()
        if self.q.grad_double_last_batch:
            user_scale, head_scale = 2.0, 1.0  # Q2: collect() doubles the last batch's grads
        else:
            user_scale = head_scale = 1.0 / n_steps
        self.flat.grad.mul_(user_scale)  # only user grads are non-zero at this point
        ids = torch.nonzero(self.touched).reshape(-1).to(torch.int32)
        te = self.model.text_encoder
        # Q4 (compat): the reference replays the text encoder in train mode (model.py:73), i.e.
        # re-runs DistilBERT with dropout on the touched titles; the default is the exact
        # eval-mode VJP over the hidden states the vectors were computed from (E10)
        train_mode = self.q.replay_train_mode
        te.train(train_mode)
        for s in range(0, ids.numel(), self.replay_chunk):
            cid = ids[s:s + self.replay_chunk]
            with obs.range("replay"):
                if train_mode:  # DistilBERT with its dropout (p = backbone.dropout / attention_dropout)
                    text = self.tokens.index_select(0, cid.long())
                    hid, mask = te.hidden(text, dropout=True), text[:, 1, :]
                    v = te.head(hid, mask)
                elif self.fused_head:  # the head VJP straight over the cache rows of the touched titles
                    v = te.head_rows(self.hcache.flat(), self._cache_ids(cid), self.tokens.shape[2], self.tokens)
                else:
                    hid, mask = self._hidden(cid)
                    v = te.head(hid, mask)
                v.backward(self.G.index_select(0, cid.long()) * head_scale)
        self.optimizer_step()
        self.G = None
        self.touched = None
        self.news_table = None

    def _next_prepared(self, it) -> Optional[Prepared]:
        """The next batch of a sampler iterator, sampled and de-duplicated ahead (None at the
        end of the epoch)."""
        if self._prep is None:
            b = next(it, None)
            return None if b is None else Prepared(self.to_device(b[0]), self.to_device(b[1]), None, None)
        with torch.cuda.stream(self._prep):  # the device sampler's kernel runs on the lookahead stream
            b = next(it, None)
        return None if b is None else self.prepare(lambda: b, held=True)

    INFLIGHT = 8  # held batches kept alive after their step was queued (bounds the host run-ahead)
    EVENT_EVERY = 4  # one end-of-step event per this many steps

    def _retire(self, pre: Optional[Prepared]) -> None:
        """Keep a held batch's lookahead tensors alive until the main stream has run its step.
        record_stream on the six tensors made the caching allocator queue six event records on
        the main stream per step when they were freed -- ~30 us of device idle between two step
        graphs (steady step 0.548 -> 0.529 ms without them; the bare replay loop,
        benchmarks/graph_seam.py, has an 8.6 us seam).  Here one event every EVENT_EVERY steps
        marks a step's end; a batch is released once INFLIGHT later steps are queued and an event
        recorded at or after its step has completed (the host then runs at most INFLIGHT steps
        ahead of the device, far more than the ~0.15 ms of host work per step needs)."""
        if pre is None or not pre.held or self._prep is None:
            return
        self._held_n += 1
        ev = None
        if self._held_n % self.EVENT_EVERY == 0:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        self._inflight.append((pre, ev))
        while len(self._inflight) > self.INFLIGHT:
            _, old = self._inflight.popleft()
            if old is None:  # covered by the next event queued after it
                old = next((e for _, e in self._inflight if e is not None), None)
            if old is not None:
                t0 = time.perf_counter()
                old.synchronize()
                self.host_wait_s += time.perf_counter() - t0

    # -------------------------------------------------------------------------------
    def train_epoch(self, max_steps: Optional[int] = None, log_every: int = 0,
                    step_hook: Optional[Callable[[int], None]] = None) -> Dict[str, float]:
        """One local epoch.  ``max_steps`` caps the batches (synchronous modes pass the
        minimum over clients so every rank issues the same collectives); ``step_hook(n)``
        runs after every step (parameter averaging every K steps)."""
        sched = self.cfg.resolved_local_update()
        t0 = time.perf_counter()
        losses, folded = [], []
        n = 0
        if sched == "per_epoch":
            self._begin_epoch_accumulate()
        it = iter(self.sampler.epoch(self.epoch))
        nxt = self._next_prepared(it)
        while True:
            pre = nxt
            if pre is None:
                break
            if sched == "per_step":
                loss = self.train_prepared(pre)
            else:
                loss = self.accumulate_step(pre.cand, pre.his, pre)
                self._retire(pre)
            # sample + dedup the next batch while this step's kernels run (both schedules)
            last = max_steps is not None and n + 1 >= max_steps
            nxt = None if last else self._next_prepared(it)
            losses.append(loss)
            if len(losses) >= self.LOSS_RING // 2:  # fold before the loss ring wraps
                folded.append(torch.stack(losses).float().sum())
                losses = []
            n += 1
            if step_hook is not None:
                self.sync_params()  # hooks (parameter averaging every K steps) read the parameters
                step_hook(n)
            if log_every and n % log_every == 0:
                obs.log(f"[rank {self.rank}] epoch {self.epoch} step {n} loss {float(loss):.4f}")
            if max_steps is not None and n >= max_steps:
                break
        if sched == "per_epoch":
            self.end_epoch_update(n)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self._inflight.clear()  # every held batch's step has completed
        dt = time.perf_counter() - t0
        self.check_data_plane()
        self.epoch += 1
        parts = folded + ([torch.stack(losses).float().sum()] if losses else [])
        sum_loss = float(torch.stack(parts).sum()) if parts else float("nan")
        mean_loss = sum_loss / n if n else float("nan")
        imps = min(n * self.cfg.batch_size, len(self.shard.train))
        self.last_stats = {"training_loss": mean_loss, "training_loss_sum": sum_loss, "steps": n,
                           "impressions": imps, "epoch_s": dt, "impressions_per_s": imps / max(dt, 1e-9)}
        return self.last_stats

    @torch.no_grad()
    def validate(self, batch_size: int = 256, limit: Optional[int] = None,
                 device_batches: Optional[bool] = None) -> Dict[str, float]:
        """Corpus-mean AUC/MRR/nDCG over the validation impressions (fix of Q9).
        ``device_batches`` (None = auto: the fused device user side with truncated histories):
        the batches are assembled and scored on the device with no host step per batch
        (:meth:`_validate_device`); False = the host-batched loop."""
        self.sync_params()
        self.model.eval()
        scores_all, losses = [], []
        # the parameters do not change during validation, so every news vector is a constant:
        # when the batches would encode more titles than the corpus holds (a full validation
        # split: >= 5 titles per impression, popular titles in every batch), encode each title
        # ONCE into a table and gather -- per-title results are the same either way (every
        # kernel computes a title's rows independently of the rest of the batch)
        n_imp = len(self.shard.valid) if limit is None else min(limit, len(self.shard.valid))
        if device_batches is None:
            device_batches = self.fused_user and self.device.type == "cuda" and not self.q.no_history_truncation
        if device_batches and n_imp > 0:
            S, loss_sum = self._validate_device(batch_size, limit, n_imp)
            return self._valid_metrics(S, loss_sum)
        table = None
        if self.news_table is not None:
            table = self.news_table
        elif (self.valid_table == "always"
              or (self.valid_table == "auto" and n_imp * (self.cfg.npratio + 1) > self.N)):
            table = self.encode_all(grad=False)
            self.model.eval()
        for cand_np, his_np in validation_batches(self.shard.valid, batch_size, self.cfg.npratio,
                                                  self.cfg.max_his_len, not self.q.no_history_truncation,
                                                  limit):
            cand, his = self.to_device(cand_np), self.to_device(his_np)
            B, C = cand.shape
            ids = _adjacent_ids(cand, his)
            if self.fused_user:  # the fused device user side, forward only (eval: no dropout)
                if table is not None:
                    v, inv = table, ids.to(torch.int32)
                else:
                    uniq, inv, _, _ = ops.dedup(ids, self.N)
                    v = self.news_vectors(uniq, grad=False)
                loss, s = self._user_loss(v, (None, inv, inv, inv), B, C, his.shape[1], False, False, his)
                losses.append(float(loss) * B)
                scores_all.append(s.float().cpu().numpy())
                continue
            if table is not None:
                rows = table.index_select(0, ids.long())
            else:
                uniq, inv, _, _ = ops.dedup(ids, self.N)
                v = self.news_vectors(uniq, grad=False)
                rows = v.index_select(0, inv.long())
            cand_v = rows[: B * C].view(B, C, -1)
            his_v = rows[B * C:].view(B, his.shape[1], -1)
            u = self.model.user_encoder(his_v, his)
            loss, s, _, _ = ops.score_ce(cand_v, u, self.score_act)
            losses.append(float(loss) * B)
            scores_all.append(s.float().cpu().numpy())
        if not scores_all:
            return {"validation_loss": float("nan"), "valid_auc": float("nan"), "valid_mrr": float("nan"),
                    "val_ndcg@5": float("nan"), "val_ndcg@10": float("nan"), "n_valid": 0}
        return self._valid_metrics(np.concatenate(scores_all, 0), sum(losses))

    def prepare_validation(self, batch_size: int = 256) -> None:
        """Build the validation split's device sampler now (its arrays go to HBM once); the
        first :meth:`validate` otherwise pays it inside the round."""
        if self.device.type == "cuda" and self.fused_user and getattr(self, "_vsampler", None) is None:
            self._vsampler = DeviceSampler(self.shard.valid, batch_size, self.device, self.cfg.npratio,
                                           self.cfg.max_his_len, truncate=True, seed=self.cfg.seed, rank=self.rank,
                                           shuffle=False)

    def _validate_device(self, batch_size: int, limit: Optional[int], n_imp: int) -> Tuple[np.ndarray, float]:
        """The validation pass with no host work per batch: the batches are assembled by the
        device sampler's validation mode (``[pos] + negs[-4:]``, client.py:158-165), the news
        vectors come from one encode of the whole table (the parameters are constant during
        validation, so every title's vector is), scores and the loss sum accumulate in device
        buffers, and ONE copy brings them back.  Same values as the host-batched path
        (``test_device_validation_matches_host_batches``)."""
        self.prepare_validation(batch_size)
        table = self.news_table if self.news_table is not None else self.encode_all(grad=False)
        self.model.eval()
        C = self.cfg.npratio + 1
        S = torch.empty(n_imp, C, dtype=torch.float32, device=self.device)
        lsum = torch.zeros((), dtype=torch.float32, device=self.device)
        s0 = 0
        for cand, his in self._vsampler.valid_batches(batch_size, limit):
            B = cand.shape[0]
            ids = _adjacent_ids(cand, his)
            loss, s = self._user_loss(table, (None, ids, ids, ids), B, C, his.shape[1], False, False, his)
            S[s0:s0 + B].copy_(s)
            lsum.add_(loss.float(), alpha=float(B))
            s0 += B
        host = torch.cat([S.reshape(-1), lsum.reshape(1)]).cpu().numpy()  # the one copy back
        return host[:-1].reshape(n_imp, C), float(host[-1])

    def _valid_metrics(self, S: np.ndarray, loss_sum: float) -> Dict[str, float]:
        m = batch_metrics(S)
        out = {"validation_loss": loss_sum / S.shape[0], "valid_auc": m["auc"], "valid_mrr": m["mrr"],
               "val_ndcg@5": m["ndcg5"], "val_ndcg@10": m["ndcg10"], "n_valid": S.shape[0],
               "last_valid_auc": m["last_auc"], "last_valid_mrr": m["last_mrr"]}
        if self.q.validate_last_only:  # Q9 compat: the reference returns the last impression's values
            out.update({"valid_auc": round(m["last_auc"], 2), "valid_mrr": round(m["last_mrr"], 2),
                        "val_ndcg@5": round(m["last_ndcg5"], 2), "val_ndcg@10": round(m["last_ndcg10"], 2)})
        return out
