"""What a step-graph boundary costs on this stack: the same body of small kernels replayed as
(a) one graph per step, back to back; (b) one graph per step preceded by an eager kernel (the
step's input launch, multi_cast, today); (c) two steps per graph.  Per-step time from
torch.cuda events over many steps; the kernel body is ~20 small elementwise launches so the
per-step device time is close to the launch-bound regime of the config-2 step's boundary."""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--kernels", type=int, default=20)
    ap.add_argument("--numel", type=int, default=1 << 20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    x = torch.randn(a.numel, device=dev)
    y = torch.zeros_like(x)
    z = torch.zeros(1 << 14, device=dev)

    def body():
        for _ in range(a.kernels):
            y.mul_(0.5).add_(x)

    s = torch.cuda.Stream(dev)
    graphs = {}
    with torch.cuda.stream(s):
        for _ in range(3):
            body()
    torch.cuda.synchronize()
    for name, reps in (("one", 1), ("two", 2)):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                body()
        graphs[name] = g
    torch.cuda.synchronize()

    def run(mode, steps):
        if mode == "graph":
            for _ in range(steps):
                graphs["one"].replay()
        elif mode == "eager+graph":
            for _ in range(steps):
                z.add_(1.0)
                graphs["one"].replay()
        elif mode == "graph2":
            for _ in range(steps // 2):
                graphs["two"].replay()
        elif mode == "eager":
            for _ in range(steps):
                body()

    out = []
    for mode in ("graph", "eager+graph", "graph2", "graph", "eager+graph", "graph2"):
        run(mode, 20)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(mode, a.steps)
        e1.record()
        torch.cuda.synchronize()
        out.append({"mode": mode, "us_per_step": round(e0.elapsed_time(e1) * 1e3 / a.steps, 2),
                    "kernels_per_step": a.kernels * 2, "numel": a.numel})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
