"""Build the in-tree HIP extension ``_C.so`` for gfx950 (no hipify, no cpp_extension JIT).

* every ``*.hip`` kernel file -> ``hipcc --offload-arch=gfx950 -O3 -c`` (no torch headers,
  seconds per file, compiled in parallel);
* ``binding.cpp`` (TORCH_LIBRARY registrations) -> host compile against torch's headers;
* link with the system linker against torch's *own* ``libamdhip64`` (rpath to torch/lib),
  so the process holds exactly one HIP runtime.

Incremental: objects are rebuilt only when a source or any ``csrc/*.h`` header is newer (the
headers carry layouts that several objects share, e.g. ``gemm_batch.h``).
Usage: ``python -m fedrec_with_pytorchdistributed_amd.csrc.build [--force] [--verbose]``.

``--sanitize`` builds ``_C_san.so`` instead: the HOST code of every file
(binding.cpp's argument checks and op glue, the IPC context table and handle plumbing of
ipc_allreduce.hip, every launcher) under AddressSanitizer + UndefinedBehaviorSanitizer, with
clang for every object so one sanitizer runtime serves them all (device code is not
instrumented: ``-Xarch_host``).  It is never loaded by default; ``tests/test_sanitize_host.py``
loads it in a child process with the ASan runtime preloaded and drives the validation paths.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
OUT = PKG / "_C.so"
BUILD = HERE / "build"
ARCH = os.environ.get("FEDREC_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found")


def _rocm() -> str:
    return os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch

    root = Path(torch.__file__).resolve().parent
    return root / "include", root / "lib", int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose: bool):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


SAN = ["-fsanitize=address", "-fsanitize=undefined"]
# binding.cpp only: no global-variable instrumentation -- its string literals were registered
# twice at load (a false odr-violation report that ASAN_OPTIONS could not silence); heap, stack
# and UB checks stay on (the .hip host objects keep the full instrumentation)
SAN_CC = ["-mllvm", "-asan-globals=0"]
OUT_SAN = PKG / "_C_san.so"


def _clangxx() -> str:
    return str(Path(_rocm()) / "lib/llvm/bin/clang++")


def asan_runtime() -> str:
    """The clang ASan runtime the sanitized build links against (LD_PRELOAD it)."""
    return subprocess.run([_clangxx(), "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True,
                          text=True).stdout.strip()


def build(force: bool = False, verbose: bool = False, jobs: int = 8, sanitize: bool = False) -> Path:
    bdir = BUILD / "san" if sanitize else BUILD
    out = OUT_SAN if sanitize else OUT
    bdir.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    tinc, tlib, abi = _torch_paths()
    common = sorted(HERE.glob("*.h"))  # every shared header: a layout change rebuilds every object
    kernels = sorted(HERE.glob("*.hip"))
    jobs_list = []
    objs = []
    # host-only sanitizers: each -fsanitize= right after -Xarch_host (device code uninstrumented)
    hsan = [a for f in SAN for a in ("-Xarch_host", f)] + ["-Xarch_host", "-fno-omit-frame-pointer"] if sanitize else []
    for src in kernels:
        obj = bdir / (src.stem + ".o")
        objs.append(obj)
        if force or _newer(obj, [src, *common]):
            jobs_list.append([hipcc, f"--offload-arch={ARCH}", "-O3" if not sanitize else "-O1", "-fPIC", "-std=c++17",
                              "-munsafe-fp-atomics", *hsan, "-c", str(src), "-o", str(obj)])
    bsrc = HERE / "binding.cpp"
    bobj = bdir / "binding.o"
    objs.append(bobj)
    if force or _newer(bobj, [bsrc, *common]):
        cxx, extra = ("g++", ["-O2"]) if not sanitize else (_clangxx(), ["-O1", *SAN, *SAN_CC,
                                                                          "-fno-omit-frame-pointer"])
        jobs_list.append([cxx, *extra, "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
                          f"-I{_rocm()}/include",
                          f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{tinc}", f"-I{tinc / 'torch/csrc/api/include'}",
                          f"-I{sysconfig.get_paths()['include']}", "-c", str(bsrc), "-o", str(bobj)])
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(jobs_list)))) as ex:
            for f in [ex.submit(_run, c, verbose) for c in jobs_list]:
                f.result()
    if force or jobs_list or _newer(out, objs):
        tmp = out.with_suffix(".so.tmp")
        link = ["g++", "-shared"] if not sanitize else [_clangxx(), "-shared", *SAN, "-shared-libsan"]
        _run([*link, "-o", str(tmp), *map(str, objs), f"-L{tlib}", "-lamdhip64", "-lc10", "-lc10_hip", "-ltorch_cpu",
              "-ltorch_hip", f"-Wl,-rpath,{tlib}"], verbose)
        os.replace(tmp, out)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--sanitize", action="store_true", help="host ASan + UBSan build -> _C_san.so")
    a = ap.parse_args(argv)
    p = build(a.force, a.verbose, a.j, a.sanitize)
    print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
