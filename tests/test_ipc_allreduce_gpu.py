"""The custom peer-to-peer all-reduce (csrc/ipc_allreduce.hip) on one MI355X: (1) W ranks of one
process played by one launch (the protocol's flags / barriers / slot parity, one-shot and
two-shot, fp32 and int32 wrap-around), against the exact sum; (2) W processes sharing the GPU
through real IPC handles exchanged over gloo, against gloo's all-reduce.  The 8-GPU xGMI run is
the driver's (bench.py reports its bus bandwidth beside RCCL's at N > 1)."""
import pytest
import torch

from launch_util import run_ranks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W", [2, 3, 4, 8])
@pytest.mark.parametrize("mode", ["one", "two"])
def test_ipc_allreduce_local_ranks(dev, W, mode):
    from fedrec_with_pytorchdistributed_amd.parallel.ipc_allreduce import LocalIpcGroup

    g = LocalIpcGroup(W, dev, cap=4 << 20, blocks=8)
    try:
        for it, n in enumerate([4, 1000, 1 << 16, 1 << 20]):
            xs = [torch.randn(n, device=dev) for _ in range(W)]
            exp = torch.stack([x.double() for x in xs]).sum(0)
            g.allreduce_(xs, mode)
            torch.cuda.synchronize()
            for x in xs:
                assert torch.allclose(x.double(), exp, rtol=1e-6, atol=1e-5), (W, mode, n)
            assert all(torch.equal(xs[0], x) for x in xs)  # bitwise-identical on every rank
            qi = [torch.randint(-(1 << 31), (1 << 31) - 1, (n,), device=dev, dtype=torch.int64).to(torch.int32)
                  for _ in range(W)]
            qe = torch.stack([q.to(torch.int64) for q in qi]).sum(0)
            qe = ((qe + (1 << 31)) % (1 << 32) - (1 << 31)).to(torch.int32)
            g.allreduce_(qi, mode)
            torch.cuda.synchronize()
            assert all(torch.equal(q, qe) for q in qi), (W, mode, n)
        assert g.status() == [0] * W
    finally:
        g.close()


def test_ipc_allreduce_local_28mb_int32_buckets(dev):
    """The secure reducer's bucket size: 28 MB of int32 (masked fixed point) per call, two-shot
    and one-shot, wrap-around sum exact and bitwise-identical on every rank."""
    from fedrec_with_pytorchdistributed_amd.parallel.ipc_allreduce import LocalIpcGroup

    W, n = 4, 7 << 20
    g = LocalIpcGroup(W, dev, cap=32 << 20, blocks=16)
    try:
        for mode in ("two", "one"):
            qi = [torch.randint(-(1 << 31), (1 << 31) - 1, (n,), device=dev, dtype=torch.int64).to(torch.int32)
                  for _ in range(W)]
            qe = torch.stack([q.to(torch.int64) for q in qi]).sum(0)
            qe = ((qe + (1 << 31)) % (1 << 32) - (1 << 31)).to(torch.int32)
            g.allreduce_(qi, mode)
            torch.cuda.synchronize()
            assert all(torch.equal(q, qe) for q in qi), mode
        assert g.status() == [0] * W
    finally:
        g.close()


@pytest.mark.parametrize("W", [2, 4])
def test_ipc_allreduce_multiprocess(W):
    import torch as _t

    if not _t.cuda.is_available():
        pytest.skip("no HIP device")
    outs = run_ranks([["tests/_ipc_worker.py"]] * W, timeout=180)
    for rc, out in outs:
        assert rc == 0, out[-2000:]
    if any("IPC_UNAVAILABLE" in out for _, out in outs):
        pytest.skip("same-device IPC refused by the runtime: " + outs[0][1][-300:])
    for _, out in outs:
        assert "IPC OK" in out, out[-2000:]
