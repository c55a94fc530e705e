"""Device idle between back-to-back HIP graph replays (torch.cuda.CUDAGraph) vs eager launches.

Per mode, 200 iterations of 20 tiny kernels each, timed with events; the per-iteration
time minus 20 x the single-kernel time is the launch / replay seam.  Run under
``rocprofv3 --kernel-trace`` to see the seams as device idle between kernels."""
import json
import sys

import torch


def timed(fn, iters=200):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters  # us per iteration


def main():
    dev = torch.device("cuda")
    x = torch.zeros(4096, device=dev)
    y = torch.zeros(4096, device=dev)
    K = 20
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            for _ in range(K):
                x.add_(1.0)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(K):
            x.add_(1.0)

    def eager():
        for _ in range(K):
            x.add_(1.0)

    def one():
        x.add_(1.0)

    def replay():
        g.replay()

    def replay_plus_eager():
        y.add_(1.0)
        g.replay()

    other = torch.cuda.Stream()
    z = torch.zeros(4096, device=dev)

    def replay_xstream():  # the engine's pattern: a lookahead-stream kernel + event, main waits
        with torch.cuda.stream(other):
            z.add_(1.0)
            ev = torch.cuda.Event()
            ev.record(other)
        torch.cuda.current_stream().wait_event(ev)
        y.add_(1.0)
        g.replay()

    done = torch.cuda.Event()
    done.record(other)

    def replay_wait_done():  # waiting on an event that completed long ago
        torch.cuda.current_stream().wait_event(done)
        y.add_(1.0)
        g.replay()

    out = {"one_kernel_us": timed(one, 2000), "eager_20_us": timed(eager), "replay_20_us": timed(replay),
           "eager1_plus_replay_20_us": timed(replay_plus_eager), "xstream_wait_replay_20_us": timed(replay_xstream),
           "done_event_wait_replay_20_us": timed(replay_wait_done)}
    out["replay_seam_us"] = out["replay_20_us"] - K * out["one_kernel_us"]
    print(json.dumps({k: round(v, 2) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
