"""Summarise rocprofv3 ``--pmc`` passes (scripts/gpu_pmc_cfg2.sh) per kernel family.

Each pass is its own run of the same short bench, so counters are joined per kernel family
(summed over that family's dispatches), not per dispatch.  Derived metrics:

* ``mfma_util``     SQ_VALU_MFMA_BUSY_CYCLES / (2.4 GHz peak clock x kernel wall time x 256 CUs
                    x 4 SIMDs): a LOWER bound (at a DVFS-lowered clock the true share is higher)
* ``gui_active_GHz`` GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time -- NOT a clock: the counter
                    window is wider than the kernel's timestamps (short kernels read 4-6 "GHz"),
                    kept only as a diagnostic and flagged ``gui_window_exceeds_kernel`` > 2.4
* ``lds_conflict``  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS-array cycle)
* ``read_TBps``     FETCH_SIZE [KB] / kernel wall time of its pass (L2-miss read traffic, which
                    includes Infinity-Cache hits: not HBM bandwidth)
* ``write_TBps``    WRITE_SIZE [KB] / kernel wall time of its pass (same caveat)

Usage: python benchmarks/pmc_summary.py gpurun_out/pmc2 > profiles/pmc_<tag>.json
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


PEAK_GHZ = 2.4  # MI355X peak engine clock


def family(name: str) -> str:
    m = re.search(r"gemm_nt_pp2_kernel<(\d)", name)
    if m:
        return {"0": "gemm_pp2 (QKV / out-proj / FFN2, bias)", "1": "gemm_pp2 + GELU (FFN1)"}.get(m.group(1), "gemm_pp2")
    for key, fam in (("head_pool_bwd", "head_pool_bwd"), ("head_pool", "head_pool"), ("upool_", "user pool"),
                     ("ln16p_kernel", "layernorm (persistent, + residual)"),
                     ("title_attn_packed_kernel", "title attention (packed)"),
                     ("gemm_nt_kernel", "gemm_nt 128x128 (text head)"),
                     ("dedup_kernel", "dedup (lookahead)"), ("sample_kernel", "sample (lookahead)"),
                     ("Cijk_", "hipBLASLt / rocBLAS"), ("user_attn", "user attention"),
                     ("pool_", "additive pool"), ("adam_kernel", "adam"),
                     ("ldp_rows_kernel", "LDP clip + Philox noise (config 4)"),
                     ("segsum_chunk_kernel", "news-grad segment sum (chunked)"),
                     ("segsum_fix_kernel", "news-grad segment sum edge fix-up"),
                     ("segsum_kernel", "news-grad segment sum")):
        if key in name:
            return fam
    # any other kernel: its name without the argument list (templates kept: they name variants)
    short = name.replace("(anonymous namespace)::", "")
    short = short[5:] if short.startswith("void ") else short
    short = short.split("(")[0]
    m = re.search(r"_GLOBAL__N_1\d+(\w+?)(I|E)", short)  # anonymous-namespace mangled names
    return m.group(1) if m else short[:80]


def load(path: str):
    per = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(dict)  # family -> dispatch -> ns
    with open(path) as f:
        for r in csv.DictReader(f):
            fam = family(r["Kernel_Name"])
            per[fam][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[fam][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per, {k: sum(v.values()) for k, v in dur.items()}, {k: len(v) for k, v in dur.items()}


def main(d: str) -> None:
    out = defaultdict(dict)
    for p in ("p1", "p2", "p3"):
        fn = os.path.join(d, f"{p}_counter_collection.csv")
        if not os.path.exists(fn):
            continue
        per, dur, n = load(fn)
        for fam, cs in per.items():
            out[fam].update(cs)
            out[fam][f"wall_ns_{p}"] = dur[fam]
            out[fam]["dispatches"] = n[fam]
    res = {}
    for fam, c in out.items():
        r = dict(c)
        w1 = c.get("wall_ns_p1", 0)
        if w1 and "GRBM_GUI_ACTIVE" in c:
            g = c["GRBM_GUI_ACTIVE"] / 8 / w1
            r["gui_active_GHz"] = round(g, 3)
            r["gui_window_exceeds_kernel"] = g > PEAK_GHZ
        if w1 and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            r["mfma_util"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (PEAK_GHZ * w1 * 256 * 4), 4)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_conflict"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
        if "FETCH_SIZE" in c and c.get("wall_ns_p2"):
            r["read_TBps"] = round(c["FETCH_SIZE"] * 1024 / c["wall_ns_p2"] / 1e3, 3)
        if "WRITE_SIZE" in c and c.get("wall_ns_p3"):
            r["write_TBps"] = round(c["WRITE_SIZE"] * 1024 / c["wall_ns_p3"] / 1e3, 3)
        res[fam] = r
    print(json.dumps(dict(sorted(res.items(), key=lambda kv: -kv[1].get("wall_ns_p1", 0))), indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc2")
