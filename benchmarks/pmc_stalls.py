"""Where the waves of each kernel family wait: two rocprofv3 ``--pmc`` passes of SQ wave-state
counters over the same short bench (scripts/gpu_r3_stalls.sh), joined per kernel family
(benchmarks/pmc_summary.family).  All SQ_WAIT_* / SQ_ACTIVE_* counters are wave-cycles (per
SIMD, units of 4 cycles, as SQ_WAVE_CYCLES), so the ratios below are shares of wave time:

* ``wait_any``       SQ_WAIT_ANY / SQ_WAVE_CYCLES: waiting on a dependency (s_waitcnt, barrier)
* ``wait_inst_any``  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES: ready but not issued (issue contention)
* ``active_lds`` / ``active_vmem`` / ``active_valu`` / ``active_any``: issuing that class
* ``wait_inst_lds``  SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES: an LDS instruction waiting to issue
* ``lds_per_mfma``   SQ_INSTS_LDS / SQ_INSTS_MFMA

Usage: python benchmarks/pmc_stalls.py gpurun_out/pmc_stalls > profiles/r3_pmc_stalls_cfg2.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import family  # noqa: E402


def main(d: str) -> None:
    per = defaultdict(lambda: defaultdict(float))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                per[family(r["Kernel_Name"])][r["Counter_Name"] + "@" + os.path.basename(path)[:2]] += float(
                    r["Counter_Value"])
    out = {}
    for fam, c in per.items():
        def get(name):
            vals = [v for k, v in c.items() if k.split("@")[0] == name]
            return vals[0] if vals else None

        def pass_of(name):
            return [k.split("@")[1] for k in c if k.split("@")[0] == name]

        row = {k.split("@")[0] + ("" if k.split("@")[0] != "SQ_WAVE_CYCLES" else "@" + k.split("@")[1]): v
               for k, v in c.items()}
        # each ratio against the SQ_WAVE_CYCLES of the pass that counted its numerator
        wc = {k.split("@")[1]: v for k, v in c.items() if k.split("@")[0] == "SQ_WAVE_CYCLES"}
        for name, key in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst_any"),
                          ("SQ_ACTIVE_INST_ANY", "active_any"), ("SQ_ACTIVE_INST_LDS", "active_lds"),
                          ("SQ_ACTIVE_INST_VMEM", "active_vmem"), ("SQ_ACTIVE_INST_VALU", "active_valu"),
                          ("SQ_WAIT_INST_LDS", "wait_inst_lds"), ("SQ_ACTIVE_INST_MISC", "active_misc")):
            v = get(name)
            ps = pass_of(name)
            w = wc.get(ps[0]) if ps else None
            if v is not None and w:
                row[key] = round(v / w, 4)
        li, mi = get("SQ_INSTS_LDS"), get("SQ_INSTS_MFMA")
        if li is not None and mi:
            row["lds_per_mfma"] = round(li / mi, 3)
        out[fam] = row
    ordered = dict(sorted(out.items(), key=lambda kv: -max([v for k, v in kv[1].items() if k.startswith("SQ_WAVE_CYCLES")] or [0])))
    json.dump(ordered, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
