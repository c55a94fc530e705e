"""Per-kernel register / LDS / occupancy table of one .hip file (hipcc's kernel-resource-usage
remarks), to check a kernel change for spills before it goes to the GPU.

    python scripts/resource_usage.py fedrec_with_pytorchdistributed_amd/csrc/text_head.hip [filter]
"""
import re
import subprocess
import sys


def main(path: str, filt: str = "") -> None:
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", path, "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.+?): (.+?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for r in rows:
        if filt and filt not in r["name"]:
            continue
        name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        print(f"{name[:90]:90s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>3} "
              f"spill={r.get('VGPRs Spill','?')} lds={r.get('LDS Size [bytes/block]','?'):>6} "
              f"occ={r.get('Occupancy [waves/SIMD]','?')}")


if __name__ == "__main__":
    main(*sys.argv[1:])
