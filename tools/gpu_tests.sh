#!/bin/bash
# GPU parity suite + smoke on the box (each step under its own limit; stops at the first failure)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
tail -5 gpurun_out/tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed $?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
