#!/bin/bash
# GPU parity suite, then the headline bench without the CPU baseline / configs[4] legs (iteration loop)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu --maxfail=5 -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -20 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python3 bench.py --no-cpu --no-pcond "$@" > gpurun_out/qbench.log 2>&1 || { tail -20 gpurun_out/qbench.log; exit 1; }
python3 - <<'PY'
import json
l = [x for x in open("gpurun_out/qbench.log") if x.startswith("{")][-1]
d = json.loads(l)
r = d["roofline"]
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "frac", round(r["frac"], 4), "launch_ms", round(r["launch_ms"], 4))
print("pass_ms", {k: round(v, 3) for k, v in r["pass_ms_per_step"].items()})
print("riccati", round(d["riccati"]["value"]), "N50", round((d.get("riccati_batch_N50") or {}).get("value", 0)), "single_qp_us", (d.get("single_qp") or {}).get("device_us_per_ip_iter"))
a = d.get("aliased") or {}
print("aliased", round(a.get("value", 0)), "per-problem layout", round((a.get("per_problem_layout") or {}).get("value", 0)))
for k, v in (("ipm", d.get("parity")), ("sv", d["riccati"].get("parity")), ("aliased", a.get("parity")),
             ("N50", (d.get("riccati_batch_N50") or {}).get("parity")), ("single", (d.get("single_qp") or {}).get("parity"))):
    if v:
        print("parity", k, "max_rel_err %.2e" % v["max_rel_err"], "kk_ret_equal", v.get("kk_ret_equal"))
PY
