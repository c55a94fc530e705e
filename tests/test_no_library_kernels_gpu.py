"""The training step runs our kernels only: a torch.profiler trace of one eager step (the
kernels a step graph captures) and one validation pass holds no vendor GEMM (rocBLAS /
hipBLASLt ``Cijk_*``), no ``at::native`` GEMM / matmul and no torch dropout -- in the default
configuration and with the ``mask_padding`` option (the masked user attention and pools)."""
import pytest
import torch
from torch.profiler import ProfilerActivity, profile

from fedrec_with_pytorchdistributed_amd.config import BackboneConfig, FedRecConfig
from fedrec_with_pytorchdistributed_amd.data.synthetic import make_client_shards
from fedrec_with_pytorchdistributed_amd.models.fedrec_model import FedRecModel
from fedrec_with_pytorchdistributed_amd.train.engine import LocalEngine

pytestmark = pytest.mark.gpu

_LIB_WORDS = ("gemm", "matmul", "dropout", "bernoulli")


def library_kernels(names):
    """Kernel names that are a vendor GEMM, or a torch GEMM / dropout kernel."""
    bad = []
    for n in names:
        low = n.lower()
        if "cijk" in low or "rocblas" in low or "hipblaslt" in low:
            bad.append(n)
        elif "at::native" in n and any(w in low for w in _LIB_WORDS):
            bad.append(n)
    return bad


def test_classifier_flags_vendor_and_torch_kernels():
    assert library_kernels(["Cijk_Alik_Bljk_BBS_BH_MT64x64", "void at::native::fused_dropout_kernel<float>",
                            "small_gemm_kernel<2, 2, true, false, true>", "user_attn_fwd_mfma4_kernel"]) == [
        "Cijk_Alik_Bljk_BBS_BH_MT64x64", "void at::native::fused_dropout_kernel<float>"]


def _kernel_names(prof):
    return [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]


@pytest.mark.parametrize("mask", [False, True])
def test_step_and_validation_use_only_our_kernels(dev, mask):
    cfg = FedRecConfig(mode="grad_avg", batch_size=16, mask_padding=mask)  # user dropout 0.2 (default)
    cfg.backbone = BackboneConfig(name="distilbert-2l", n_layers=2)
    torch.manual_seed(0)
    m = FedRecModel(cfg).to(dev)
    m.build_flat()
    eng = LocalEngine(cfg, m, make_client_shards("tiny", 1)[0], dev)
    assert eng.fused_user
    batches = [tuple(eng.to_device(a) for a in b) for _, b in zip(range(2), eng.sampler.epoch(0))]
    eng.train_step(*batches[0])  # first-call setup (caches, casts) outside the trace
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        loss = eng.train_step(*batches[1])
        eng.validate(limit=32)
        torch.cuda.synchronize()
    names = _kernel_names(prof)
    assert torch.isfinite(loss)
    assert len(names) > 20, "the profiler saw no kernels"
    assert any("small_gemm" in n for n in names) and any("user_attn" in n for n in names)
    bad = library_kernels(names)
    assert not bad, sorted(set(bad))


def test_default_text_head_kernels(dev):
    """The default step runs the staged-wait form of head_score2 (SW = true) and the G path of the
    backward (head_pool_bwd3: the pool backward with the g rewrite in the same launch, then the
    plain TN GEMM head_wgrad_g -- not the round-4 head_wgrad with its in-pipeline rewrite, nor the
    separate head_g_rewrite launch): guards the defaults of csrc/text_head.hip / ops.functional."""
    cfg = FedRecConfig(mode="grad_avg", batch_size=16)  # the headline backbone (Q = 384 head)
    torch.manual_seed(0)
    m = FedRecModel(cfg).to(dev)
    m.build_flat()
    eng = LocalEngine(cfg, m, make_client_shards("tiny", 1)[0], dev)
    if not eng.fused_head:
        pytest.skip("this configuration does not take the fused text head")
    batches = [tuple(eng.to_device(a) for a in b) for _, b in zip(range(2), eng.sampler.epoch(0))]
    eng.train_step(*batches[0])
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        eng.train_step(*batches[1])
        torch.cuda.synchronize()
    names = _kernel_names(prof)
    hs = [n for n in names if "head_score2_kernel" in n]
    wg = [n for n in names if "head_wgrad_g_kernel" in n]
    gr = [n for n in names if "head_pool_bwd3_kernel" in n]
    assert hs and wg and gr, sorted(set(n for n in names if "head" in n))
    assert not [n for n in names if "head_g_rewrite_kernel" in n]  # fused into head_pool_bwd3
    assert not [n for n in names if "head_wgrad_kernel" in n]  # the round-4 form is off by default
    # bool template arguments: mangled "Lb1E" or demangled "true>" (the last template argument)
    assert all("Lb1EE" in n or n.split(">")[0].rstrip().endswith("true") for n in hs), sorted(set(hs))
