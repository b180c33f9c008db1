#!/bin/bash
# quick GPU iteration: parity suite, per-kernel timings, optional stamp breakdown
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x > gpurun_out/tests.log 2>&1; rc=$?
tail -5 gpurun_out/tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/tests.log | head -20; exit $rc; }
timeout -k 10 300 python3 tools/ubench.py > gpurun_out/ubench.log 2>&1 || { echo "ubench failed $?"; tail -20 gpurun_out/ubench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ubench.log
if [ "$1" == "stamps" ]; then
  timeout -k 10 300 python3 tools/stamps.py > gpurun_out/stamps.log 2>&1 || { echo "stamps failed $?"; tail -20 gpurun_out/stamps.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps.log
fi
