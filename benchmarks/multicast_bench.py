"""What the step's input launch (csrc/adam.hip multi_cast: the step's weight casts + the batch
copy) spends its ~8 us on: the config-2 weight casts as the step issues them, without the
transposed segment (W1^T of the user pool), the transposed segment with one tiny plain one (a launch needs one),
and one tiny segment
(the launch floor).  Each form is captured 20 times back to back in one HIP graph (no graph
boundary per launch), replayed, and timed per launch."""
import json

import torch

from fedrec_with_pytorchdistributed_amd.config import FedRecConfig
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
from fedrec_with_pytorchdistributed_amd.ops import functional as OF
from fedrec_with_pytorchdistributed_amd.ops import native


def main():
    dev = torch.device("cuda", 0)
    cfg = FedRecConfig(mode="grad_avg")
    model = FedRecModel(cfg).to(dev)
    te, ue = model.text_encoder, model.user_encoder
    bufs = OF.step_cast_buffers(te, ue)
    src, dst = OF.step_cast_lists(te, ue, bufs)
    lib = native.lib()
    tmask = [d.dim() == 2 and d.stride(0) == 1 and d.stride(1) != 1 for d in dst]  # transposed views
    tiny_s, tiny_d = torch.randn(64, device=dev), torch.empty(64, device=dev)
    forms = {
        "all (as the step)": (src, dst),
        "without the transposed segment": ([s for s, t in zip(src, tmask) if not t], [d for d, t in zip(dst, tmask) if not t]),
        "transposed segment + one 64-element segment": ([tiny_s] + [s for s, t in zip(src, tmask) if t],
                                                        [tiny_d] + [d for d, t in zip(dst, tmask) if t]),
        "one 64-element segment": ([tiny_s], [tiny_d]),
    }
    out = []
    for name, (s, d) in forms.items():
        if not s:
            continue
        assert lib.multi_cast(s, d)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                lib.multi_cast(s, d)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 400
        out.append({"form": name, "segments": len(s), "elements": int(sum(t.numel() for t in s)),
                    "us_per_launch": round(us, 2)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
