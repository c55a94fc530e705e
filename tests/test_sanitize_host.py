"""the extension's HOST code under AddressSanitizer + UndefinedBehaviorSanitizer.

``csrc/build.py --sanitize`` builds ``_C_san.so`` (clang for every object, ``-fsanitize`` on
the host side only); a child process loads it with the ASan runtime preloaded and drives:

* the op registration (every ``TORCH_LIBRARY`` schema parses; the library initialisers run);
* ``binding.cpp``'s argument validation: ops called with host tensors, wrong dtypes, wrong
  sizes and empty lists must raise ``RuntimeError`` from their checks (no out-of-bounds read of
  a tensor list, no signed overflow in a size computation) -- the CPU container has no device,
  so the checks are the code that runs;
* the IPC all-reduce's host context table (``ipc_allreduce.hip``): bad ids, out-of-range
  ranks / world sizes, a context create that fails (no device) -- error codes, never a
  stray write into the 64-slot table.

A sanitizer report makes the child exit non-zero (``halt_on_error``); the test fails on it."""
import os
import subprocess
import sys

import pytest

from launch_util import ROOT

CHILD = r'''
import sys, torch
torch.ops.load_library(sys.argv[1])
F = torch.ops.fedrec
n_ok = 0

def raises(fn, *a, **k):
    global n_ok
    try:
        fn(*a, **k)
    except (RuntimeError, TypeError, ValueError):
        n_ok += 1
        return
    raise AssertionError(f"{fn} accepted bad arguments")

x = torch.zeros(8, 4)
i32 = torch.zeros(8, dtype=torch.int32)
bf = torch.zeros(8, 4, dtype=torch.bfloat16)
# host tensors where device tensors are required, wrong dtypes / shapes, empty lists
raises(F.adam_flat, x, x, x, x, 1, 1e-3, 0.9, 0.999, 1e-8, 1.0)
raises(F.multi_cast, [x], [])
raises(F.multi_cast, [], [x])
raises(F.multi_copy, [x, x], [x], [0, 0])
raises(F.head_pool_bwd, bf, None, 50, x, x, None)
raises(F.head_wgrad_g, bf, None, 50, bf, x, x.reshape(-1), x.reshape(-1), None)
raises(F.segment_sum_rows, x, i32, i32, 7, 0.0, 0.0, 0, 0, None, False, None)
raises(F.ipc_allreduce_, 0, x.reshape(-1), 1, 0, 8, 1.0)
raises(F.ipc_allreduce_local_, [0, 1], [x.reshape(-1)], 1, 0, 8, 1.0)
raises(F.ipc_allreduce_local_, list(range(17)), [x.reshape(-1)] * 17, 1, 0, 8, 1.0)
raises(F.ipc_open, 0, torch.zeros(64, dtype=torch.uint8), 0, 2, None)      # handles of W=1, W=2 asked
raises(F.ipc_open, 0, torch.zeros(128, dtype=torch.int32), 0, 2, None)     # wrong dtype
raises(F.ipc_open, 70, torch.zeros(128, dtype=torch.uint8), 0, 2, None)    # id past the table
raises(F.ipc_open, -3, torch.zeros(128, dtype=torch.uint8), 0, 2, None)
raises(F.ipc_open, 0, torch.zeros(64 * 17, dtype=torch.uint8), 0, 17, None)  # W past MAXW
raises(F.ipc_open, 0, torch.zeros(128, dtype=torch.uint8), 5, 2, None)     # rank past W
raises(F.ipc_status, 99)
raises(F.ipc_status, -1)
raises(F.ipc_create, 17)         # capacity not a multiple of 16
raises(F.ipc_create, 1 << 20)    # no device here: the allocation fails cleanly
for bad in (-1, 64, 1000):
    F.ipc_destroy(bad)           # out-of-range ids are ignored
assert F.ipc_region(5) == 0 and F.ipc_region(-2) == 0
print(f"SANITIZED OK {n_ok}", flush=True)
'''


@pytest.mark.slow
def test_host_code_under_asan_ubsan(tmp_path):
    sys.path.insert(0, ROOT)
    from fedrec_with_pytorchdistributed_amd.csrc import build as b

    so = b.build(sanitize=True)
    rt = b.asan_runtime()
    assert os.path.exists(rt), rt
    env = dict(os.environ)
    env.update({"LD_PRELOAD": rt,
                "ASAN_OPTIONS": "detect_leaks=0:alloc_dealloc_mismatch=0:detect_odr_violation=0:halt_on_error=1:"
                                "abort_on_error=0:exitcode=86",
                "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1:exitcode=87",
                "HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": ""})
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    r = subprocess.run([sys.executable, str(script), str(so)], env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "SANITIZED OK" in out and "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    n = int(out.split("SANITIZED OK")[1].split()[0])
    assert n >= 20
