#!/usr/bin/env python3
"""Fold the instruction-mix / stall counter passes of tools/pmc_mix.sh into one JSON per kernel.

SQ_WAVE_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md, rocprofv3 PMC); the derived
fractions are ratios of the same unit.  SQ_VALU_MFMA_BUSY_CYCLES counts cycles; SQ_BUSY_CYCLES is the SQ-busy
cycle count summed over the SEs, so MFMA busy is reported per CU-cycle with GRBM_GUI_ACTIVE (summed over the 8
XCDs) as the clock: mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main(root, out):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                kn = row.get("Kernel_Name", "")
                m = re.search(r"(hk_[a-z0-9_]+)", kn)
                if not m:
                    continue
                name = m.group(1)
                sh = re.search(r"FixSh<(\d+), *(\d+)>", kn)
                if name == "hk_ric_sv" and sh and sh.groups() != ("4", "12"):
                    name += f"_nu{sh.group(1)}_nx{sh.group(2)}"  # configs[2]'s instance
                vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {"method": "rocprofv3 --pmc, one pass per counter group (tools/pmc_mix.sh) over tools/pmc_run.py; "
                     "values are per-launch means", "kernels": {}}
    for k, cs in sorted(vals.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = dict(launches=max(len(v) for v in cs.values()), per_launch=m)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in m:
                    d[c.lower().replace("sq_", "") + "_frac_of_wave_cycles"] = m[c] / wc
        if "SQ_INSTS_VALU" in m and "SQ_INSTS_SALU" in m:
            tot = m["SQ_INSTS_VALU"] + m["SQ_INSTS_SALU"] + m.get("SQ_INSTS_VMEM", 0.0) + m.get("SQ_INSTS_LDS", 0.0)
            d["valu_share_of_instructions"] = m["SQ_INSTS_VALU"] / tot if tot else None
        if "SQ_INSTS_MFMA" in m and "SQ_INSTS_VALU" in m and m["SQ_INSTS_VALU"]:
            d["mfma_share_of_valu"] = m["SQ_INSTS_MFMA"] / m["SQ_INSTS_VALU"]
        f64 = [m.get(c) for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                  "SQ_INSTS_VALU_TRANS_F64")]
        if all(x is not None for x in f64):
            d["f64_valu_instructions"] = sum(f64)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m and m["GRBM_GUI_ACTIVE"]:
            simd_cycles = m["GRBM_GUI_ACTIVE"] / 8.0 * 256 * 4
            d["mfma_busy_frac_of_simd_cycles"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
        if "TA_TA_BUSY_sum" in m and "GRBM_GUI_ACTIVE" in m and m["GRBM_GUI_ACTIVE"]:
            d["ta_busy_frac_of_cu_cycles"] = m["TA_TA_BUSY_sum"] / (m["GRBM_GUI_ACTIVE"] / 8.0 * 256)
        res["kernels"][k] = d
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, d in res["kernels"].items():
        print(k, {a: (round(b, 4) if isinstance(b, float) else b) for a, b in d.items() if a != "per_launch"})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
