#!/bin/bash
# A/B timing of two (or more: AB_VARIANTS="A B C") builds of the library on ONE box: hpmpc_amd/lib/ab/lib<v>.so
# (copies of the in-tree build before / after a change), loaded through HPMPC_MI355X_LIB by alternating runs, so
# box-to-box variance (+-5-10 % between boxes) does not decide the comparison.  The parity suite runs first, on the in-tree
# build (AB_SKIP_TESTS=1 skips it).  Every GPU step has its own time limit; the script stops at the first failure.
#   tools/gpu_ab.sh            headline queue runs (bench.py, no CPU / configs[4] legs)
#   tools/gpu_ab.sh latency    lone-QP latency (tools/latency_probe.py)
#   tools/gpu_ab.sh ric        headline runs with the isolated legs (configs[2] Riccati, the lone QP) included
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
mode=${1:-headline}
if [ "${AB_SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -20 gpurun_out/tests.log; exit 1; }
  tail -1 gpurun_out/tests.log
fi
for i in 1 2 3; do
  for v in ${AB_VARIANTS:-A B}; do
    if [ "$mode" = latency ]; then
      HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/lib$v.so timeout -k 10 300 python3 tools/latency_probe.py \
        > gpurun_out/ab/lat_$v$i.log 2>&1 || { tail -20 gpurun_out/ab/lat_$v$i.log; exit 1; }
      echo "$v$i $(grep -E 'solo' gpurun_out/ab/lat_$v$i.log)"
      continue
    fi
    iso=--no-isolated
    [ "$mode" = ric ] && iso=  # the Riccati legs: configs[2] (riccati_batch_N50) runs with the isolated legs
    HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/lib$v.so timeout -k 10 300 python3 bench.py --no-cpu --no-pcond $iso \
      --no-queue-batch-slots --no-aliased --steps 20 > gpurun_out/ab/$v$i.log 2>&1 || { tail -20 gpurun_out/ab/$v$i.log; exit 1; }
    python3 - "$v$i" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/ab/{sys.argv[1]}.log") if x.startswith("{")][-1]
d = json.loads(l)
p = d["roofline"]["pass_ms_per_step"]
par = d.get("parity") or {}
print(sys.argv[1], round(d["value"]), {k[7:]: round(v, 3) for k, v in p.items()}, "ric", round(d["riccati"]["value"]),
      "N50", round((d.get("riccati_batch_N50") or {}).get("value", 0)), "parity", par.get("max_rel_err"),
      par.get("kk_ret_equal"))
PY
  done
done
