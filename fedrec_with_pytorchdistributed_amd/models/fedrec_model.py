"""The federated model container (reference ``UserModel``, ``model.py:10-129``).

Holds ``text_encoder`` + ``user_encoder`` in registration order, so ``state_dict()`` has
exactly the reference's 116 keys (E2), and lays every *trainable* parameter out in one
contiguous fp32 buffer (:class:`FlatParams`): parameters, gradients and both Adam moments
are flat, so the gradient all-reduce is one RCCL call over one bucket and Adam is one
kernel (replacing the reference's two ``torch.optim.Adam`` instances, ``model.py:22-23``,
which always step together in ``update()``, ``model.py:66-70``).

Trainable set (frozen backbone, ``model.py:25-26``): text head 603,281 + user encoder
561,601 = 1,164,882 params in 16 tensors (4.66 MB fp32).  With
``backbone.frozen=False`` (BASELINE config 5) the backbone joins the flat store.
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Tuple

import torch
from torch import nn

from ..config import FedRecConfig
from .encoders import TextEncoder, UserEncoder


class FlatParams:
    """Parameters re-pointed into one flat fp32 buffer (+ flat grad, Adam m/v)."""

    ALIGN = 64  # elements; keeps every view 256-B aligned for vector loads

    def __init__(self, named: List[Tuple[str, nn.Parameter]]):
        self.names = [n for n, _ in named]
        self.params = [p for _, p in named]
        offs, o = [], 0
        for p in self.params:
            offs.append(o)
            o += -(-p.numel() // self.ALIGN) * self.ALIGN
        self.offsets = offs
        self.numel_padded = o
        self.numel = sum(p.numel() for p in self.params)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.zeros(o, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(o, dtype=torch.float32, device=dev)
        self.m = torch.zeros(o, dtype=torch.float32, device=dev)
        self.v = torch.zeros(o, dtype=torch.float32, device=dev)
        self.step = 0
        with torch.no_grad():
            for p, off in zip(self.params, offs):
                n = p.numel()
                self.flat[off:off + n].copy_(p.detach().reshape(-1).float())
                p.data = self.flat[off:off + n].view_as(p)
                p.grad = self.grad[off:off + n].view_as(p)

    def views(self) -> Iterator[Tuple[str, torch.Tensor, int]]:
        for n, p, off in zip(self.names, self.params, self.offsets):
            yield n, p, off

    def zero_grad(self) -> None:
        self.grad.zero_()
        # autograd may have replaced .grad (e.g. set_to_none elsewhere): re-point
        for p, off in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[off:].data_ptr():
                p.grad = self.grad[off:off + p.numel()].view_as(p)

    def begin_backward(self) -> None:
        """Detach ``.grad`` so autograd hands over fresh gradient tensors instead of
        accumulating into the flat views one add kernel per parameter."""
        for p in self.params:
            p.grad = None

    def end_backward(self, copy: bool = True, inplace=()):
        """Gather the fresh gradients into the flat buffer (one multi-tensor copy launch;
        parameters that got no gradient are zeroed) and re-point ``.grad`` at it.

        ``copy=False`` (the in-graph Adam, which gathers them itself -- csrc/adam.hip gradient
        segments): no copy launch; returns each parameter's gradient source in parameter
        order -- the fresh tensor, its flat slot when the gradient already sits there, or None
        (no gradient: Adam writes zeros) -- for the caller to hand to Adam, which writes them
        into the flat buffer.  The caller keeps the list alive until Adam is queued.

        ``inplace``: ids of parameters whose gradients the backward wrote straight into their
        slots (``ops.functional.grads_into``, N > 1): present, not missing."""
        if not copy:
            srcs = []
            for p, off in zip(self.params, self.offsets):
                view = self.grad[off:off + p.numel()].view_as(p)
                gr = view if p.grad is None and id(p) in inplace else p.grad
                if gr is not None and gr.data_ptr() != view.data_ptr() and (gr.dtype != torch.float32
                                                                           or not gr.is_contiguous()):
                    view.copy_(gr)  # (not expected on the fused step: every gradient is fresh fp32)
                    gr = view
                srcs.append(gr)
                p.grad = view
            return srcs
        dst, src, missing = [], [], []
        for p, off in zip(self.params, self.offsets):
            view = self.grad[off:off + p.numel()].view_as(p)
            if p.grad is None and id(p) in inplace:
                pass  # already in its slot
            elif p.grad is None:
                missing.append(view)
            elif p.grad.data_ptr() != view.data_ptr():
                dst.append(view)
                src.append(p.grad)
            p.grad = view
        if dst and not missing and self.grad.is_cuda and all(t.is_contiguous() and t.dtype == torch.float32
                                                              for t in src):
            # every fresh gradient into its slot in one copy launch (csrc/adam.hip multi_cast; the
            # alignment gaps are never written and stay zero; slots already holding their
            # gradient -- the early-reduced user slice at N > 1 -- are skipped); torch.cat of the
            # 110M config-5 gradients took ~0.58 ms per step in ~15 launches
            from ..ops import native
            if native.lib().multi_cast(src, dst):
                return
        if dst and not missing and len(dst) == len(self.params):
            # every parameter has a fresh gradient: one cat of [grad, zero gap, grad, ...] into
            # the flat buffer (a single batched copy kernel; the multi-tensor copy took ~18 us
            # for these 4.66 MB).  The alignment gaps get zeros, as the buffer was created.
            if getattr(self, "_cat_parts", None) is None or self._cat_parts[0] != self.grad.device:
                gaps = []
                for i, (p, off) in enumerate(zip(self.params, self.offsets)):
                    end = self.offsets[i + 1] if i + 1 < len(self.offsets) else self.numel_padded
                    gaps.append(end - off - p.numel())
                self._cat_parts = (self.grad.device,
                                   [torch.zeros(g, device=self.grad.device) if g > 0 else None for g in gaps])
            parts = []
            for t, z in zip(src, self._cat_parts[1]):
                parts.append(t.reshape(-1))
                if z is not None:
                    parts.append(z)
            torch.cat(parts, out=self.grad)
            return
        if dst:
            torch._foreach_copy_(dst, src)
        if missing:
            torch._foreach_zero_(missing)

    def state(self) -> Dict[str, torch.Tensor]:
        return {"m": self.m.detach().cpu(), "v": self.v.detach().cpu(), "step": torch.tensor(self.step)}

    def load_state(self, s: Dict[str, torch.Tensor]) -> None:
        self.m.copy_(s["m"].to(self.m.device))
        self.v.copy_(s["v"].to(self.v.device))
        self.step = int(s["step"])


class FedRecModel(nn.Module):
    def __init__(self, cfg: FedRecConfig):
        super().__init__()
        self.cfg = cfg
        self.text_encoder = TextEncoder(cfg)
        self.user_encoder = UserEncoder(cfg)
        if cfg.backbone.frozen:
            for p in self.text_encoder.DistillBert.parameters():
                p.requires_grad_(False)
        self.flat: FlatParams | None = None

    # -------------------------------------------------------------------------------
    def trainable_named(self) -> List[Tuple[str, nn.Parameter]]:
        return [(n, p) for n, p in self.named_parameters() if p.requires_grad]

    def build_flat(self) -> FlatParams:
        """Call after moving the model to its device."""
        self.flat = FlatParams(self.trainable_named())
        return self.flat

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        # copy in place so the flat views stay attached
        res = super().load_state_dict(state_dict, strict=strict, assign=False)
        self.text_encoder.DistillBert.invalidate()
        return res

    def num_params(self) -> Tuple[int, int]:
        tot = sum(p.numel() for p in self.parameters())
        tr = sum(p.numel() for p in self.parameters() if p.requires_grad)
        return tot, tr

    def sync_tensors(self, full: bool) -> List[torch.Tensor]:
        """What a round broadcast/average moves: the flat trainable buffer, or (``sync=full``,
        Q15) every parameter like the reference (``server.py:76-77``)."""
        if not full:
            return [self.flat.flat] if self.flat is not None else [p.data for p in self.parameters() if p.requires_grad]
        out = []
        if self.flat is not None:
            out.append(self.flat.flat)
        out += [p.data for p in self.parameters() if not p.requires_grad]
        return out
