"""Build the in-tree HIP extension ``_C.so`` for gfx950 (no hipify, no cpp_extension JIT).

* every ``*.hip`` kernel file -> ``hipcc --offload-arch=gfx950 -O3 -c`` (no torch headers,
  seconds per file, compiled in parallel);
* ``binding.cpp`` (TORCH_LIBRARY registrations) -> host compile against torch's headers;
* link with the system linker against torch's *own* ``libamdhip64`` (rpath to torch/lib),
  so the process holds exactly one HIP runtime.

Incremental: objects are rebuilt only when a source or ``common.h`` is newer.
Usage: ``python -m fedrec_with_pytorchdistributed_amd.csrc.build [--force] [--verbose]``.
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


def build(force: bool = False, verbose: bool = False, jobs: int = 8) -> Path:
    BUILD.mkdir(exist_ok=True)
    hipcc = _hipcc()
    tinc, tlib, abi = _torch_paths()
    common = [HERE / "common.h"]
    kernels = sorted(HERE.glob("*.hip"))
    jobs_list = []
    objs = []
    for src in kernels:
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _newer(obj, [src, *common]):
            jobs_list.append([hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
                              "-c", str(src), "-o", str(obj)])
    bsrc = HERE / "binding.cpp"
    bobj = BUILD / "binding.o"
    objs.append(bobj)
    if force or _newer(bobj, [bsrc]):
        jobs_list.append(["g++", "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
                          f"-I{_rocm()}/include",
                          f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{tinc}", f"-I{tinc / 'torch/csrc/api/include'}",
                          f"-I{sysconfig.get_paths()['include']}", "-c", str(bsrc), "-o", str(bobj)])
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(jobs_list)))) as ex:
            for f in [ex.submit(_run, c, verbose) for c in jobs_list]:
                f.result()
    if force or jobs_list or _newer(OUT, objs):
        tmp = OUT.with_suffix(".so.tmp")
        _run(["g++", "-shared", "-o", str(tmp), *map(str, objs), f"-L{tlib}", "-lamdhip64", "-lc10", "-lc10_hip",
              "-ltorch_cpu", "-ltorch_hip", f"-Wl,-rpath,{tlib}"], verbose)
        os.replace(tmp, OUT)
    return OUT


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args(argv)
    p = build(a.force, a.verbose, a.j)
    print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
