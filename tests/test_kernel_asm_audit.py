"""Static checks on the gfx950 machine code of every kernel file (CPU: hipcc cross-compiles).

* No scratch: a kernel that spills to private memory issues scratch loads, which are VMEM
  operations -- they break the counted ``s_waitcnt vmcnt(N)`` waits the LDS-DMA pipelines rely
  on (round 6: a staging lambda that kept its piece pointers in private memory made head_wgrad_g
  read stages that had not landed).  Every kernel's ``.private_segment_fixed_size`` is 0 but
  for a short, bounded list of known spills outside such pipelines (SPILL_OK).
* No in-flight aliasing inside an inline-asm block: when one asm statement issues several loads,
  a later instruction of the same statement must not read a register an earlier load of it is
  still writing (round 6: ``tr_read2`` lacked an early-clobber output, and the compiler gave the
  first ``ds_read_b64_tr_b16`` the address register the second read still needed -- wrong LDS
  rows whenever the first read returned before the queued second one issued).
"""
import concurrent.futures as cf
import re
import shutil
import subprocess
from pathlib import Path

import pytest

CSRC = Path(__file__).resolve().parents[1] / "fedrec_with_pytorchdistributed_amd" / "csrc"
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if Path("/opt/rocm/bin/hipcc").exists() else None)

pytestmark = pytest.mark.skipif(HIPCC is None, reason="hipcc not available")

_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
# loads whose FIRST operand is a vector destination written when the data returns
_LOAD = re.compile(r"^(ds_read|ds_load|global_load(?!_lds)|buffer_load(?!.*\blds\b)|flat_load|scratch_load)")


def _regs(text):
    out = set()
    for kind, lo, hi, one in _REG.findall(text):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


def _device_asm(src: Path, tmp: Path) -> str:
    out = tmp / (src.stem + ".s")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
                    "--cuda-device-only", "-S", str(src), "-o", str(out)], check=True, capture_output=True)
    return out.read_text()


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("asm")
    srcs = sorted(CSRC.glob("*.hip"))
    with cf.ThreadPoolExecutor(max_workers=6) as ex:
        texts = list(ex.map(lambda s: _device_asm(s, tmp), srcs))
    return dict(zip((s.name for s in srcs), texts))


def test_every_kernel_file_compiles_and_has_kernels(asm):
    assert len(asm) >= 15
    n = sum(len(re.findall(r"^\s*\.amdhsa_kernel ", t, re.M)) for t in asm.values())
    assert n >= 50, n


# Known spills, none in an LDS-DMA pipeline with counted waits (plain loads, compiler-managed
# waits): the value is the byte count they may not exceed.
#  * the generic small GEMM (any alignment / per-desc dtypes; no default path launches it);
#  * the title attention variants that trade a little spill for occupancy or prefetch depth
#    (title_attn.hip: the 2-waves/SIMD persistent form; title_attn_bwd.hip: the dropout
#    backward's Philox keep words -- 68 B in the default split-prefetch form, 432 B in the other).
SPILL_OK = {
    "small_gemm_kernelILi2ELi2ELb0ELb0ELb0ELb0ELb0E": 1176,
    "title_attn_pkernelILi2ELi1ELb0E": 116,
    "title_attn_bwd_pkernelILb0ELb0E": 116,
    "title_attn_bwd_pkernelILb1ELb1E": 68,
    "title_attn_bwd_pkernelILb1ELb0E": 432,
}


def test_no_kernel_uses_scratch(asm):
    bad = []
    for name, text in asm.items():
        for kern, body in re.findall(r"^\s*\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", text, re.M | re.S):
            m = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", body)
            used = int(m.group(1)) if m else 0
            limit = next((v for k, v in SPILL_OK.items() if k in kern), 0)
            if used > limit:
                bad.append((name, kern[:90], used))
    assert not bad, bad


def _aliasing(block: str):
    """Instructions of one inline-asm block that touch a register an earlier load of the block
    may still be writing (no s_waitcnt in between)."""
    bad, inflight = [], set()
    for line in block.splitlines():
        ins = line.split(";")[0].strip()
        if not ins:
            continue
        if ins.startswith("s_waitcnt"):
            inflight.clear()  # conservative: any wait in the block settles the tracking
            continue
        op, _, rest = ins.partition(" ")
        operands = [o.strip() for o in rest.split(",")]
        if _LOAD.match(op) and operands:
            if _regs(",".join(operands[1:])) & inflight:
                bad.append(ins)
            inflight |= _regs(operands[0])
        elif _regs(rest) & inflight:
            bad.append(ins)
    return bad


def test_alias_checker_flags_the_round6_pattern():
    # what the compiler emitted for tr_read2 without the early-clobber output
    assert _aliasing("ds_read_b64_tr_b16 v[98:99], v98\nds_read_b64_tr_b16 v[100:101], v98 offset:1024\n")
    assert not _aliasing("ds_read_b64_tr_b16 v[98:99], v105\nds_read_b64_tr_b16 v[100:101], v105 offset:1024\n")
    assert not _aliasing("ds_read_b32 v140, v129\ns_waitcnt lgkmcnt(0)\nv_add_u32 v1, v140, v2\n")


def test_inline_asm_loads_do_not_alias_later_operands(asm):
    bad, blocks = [], 0
    for name, text in asm.items():
        for block in re.findall(r";;#ASMSTART\n(.*?);;#ASMEND", text, re.S):
            blocks += 1
            bad += [(name, ins) for ins in _aliasing(block)]
    assert blocks > 20
    assert not bad, bad[:10]
