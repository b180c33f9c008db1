#!/usr/bin/env python3
"""Fold rocprofv3 --pmc counter CSVs into profiles/pmc_hk_ipm.json.

FETCH_SIZE / WRITE_SIZE are scaled by the factors measured on calib_copy (known bytes: 1 GiB read,
1 GiB written per launch, same 8-byte raw-buffer access width as the solver kernels)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def read_counters(d):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                c = row.get("Counter_Name", "")
                v = float(row.get("Counter_Value", "nan"))
                m = re.search(r"(hk_[a-z_]+|calib_copy)", k)
                name = m.group(1) if m else k.split("(")[0].strip()
                sh = re.search(r"FixSh<(\d+), *(\d+)>", k)
                if name == "hk_ric_sv" and sh and sh.groups() != ("4", "12"):
                    name += f"_nu{sh.group(1)}_nx{sh.group(2)}"  # configs[2]'s instance beside the headline shape
                vals[name][c].append(v)
    return vals


def main(fetch_dir, write_dir, out, kk_sum):
    F, W = read_counters(fetch_dir), read_counters(write_dir)
    known = float(1 << 30)
    cf = known / (sum(F["calib_copy"]["FETCH_SIZE"]) / len(F["calib_copy"]["FETCH_SIZE"]))
    cw = known / (sum(W["calib_copy"]["WRITE_SIZE"]) / len(W["calib_copy"]["WRITE_SIZE"]))
    res = {"workload": "ipm_queue_N100_nx12_nu4_batch1024_slots8192",
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/gpu_round.sh); "
                     "per-launch values scaled by the calib_copy factors (1 GiB known bytes, 8-B/lane buffer ops)",
           "calib": {"fetch_factor": cf, "write_factor": cw,
                     "raw_fetch": F["calib_copy"]["FETCH_SIZE"], "raw_write": W["calib_copy"]["WRITE_SIZE"]},
           "kernels": {}}
    for k in ("hk_ipm_fact", "hk_ipm_pred", "hk_ipm_corr", "hk_ipm_predcorr", "hk_ipm_update", "hk_ipm_qdrain_mw", "hk_ric_sv",
              "hk_ric_sv_nu3_nx8", "hk_pcond", "hk_wide_sv", "hk_pexpand"):
        if k not in F or k not in W:
            continue
        fr = F[k]["FETCH_SIZE"]
        wr = W[k]["WRITE_SIZE"]
        fb = sum(fr) / len(fr) * cf
        wb = sum(wr) / len(wr) * cw
        res["kernels"][k] = {"raw_fetch": fr, "raw_write": wr, "fetch_bytes_per_launch": fb,
                             "write_bytes_per_launch": wb, "hbm_bytes_per_launch": fb + wb}
    ipm = [k for k in res["kernels"] if k.startswith("hk_ipm_") and k != "hk_ipm_qdrain_mw"]
    if ipm and kk_sum:
        # pmc_run.py runs the same queue twice; kk_sum is per run and counts the iterations the pass kernels ran
        # (the drained tail's iterations are the multi-wave drain's, whose bytes are reported on their own)
        tot = sum(sum(F[k]["FETCH_SIZE"]) * cf + sum(W[k]["WRITE_SIZE"]) * cw for k in ipm) / 2.0
        res["kk_sum_per_solve"] = kk_sum
        res["hbm_bytes_per_ip_iter_problem"] = tot / kk_sum
        fact = res["kernels"].get("hk_ipm_fact")
        if fact:
            res["fact_hbm_bytes_per_problem_iter"] = (sum(F["hk_ipm_fact"]["FETCH_SIZE"]) * cf +
                                                      sum(W["hk_ipm_fact"]["WRITE_SIZE"]) * cw) / 2.0 / kk_sum
    if "hk_ric_sv" in res["kernels"]:
        res["sv_hbm_bytes_per_launch"] = res["kernels"]["hk_ric_sv"]["hbm_bytes_per_launch"]
    if "hk_ric_sv_nu3_nx8" in res["kernels"]:
        res["sv_configs2_hbm_bytes_per_launch"] = res["kernels"]["hk_ric_sv_nu3_nx8"]["hbm_bytes_per_launch"]
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 0)
