#!/bin/bash
# wide-stage parity on the box: the existing wide Riccati / condensing tests (refactored kernels), then the
# wide IPM tests, then the goldens on the wide path.  Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 600 python3 -u -m pytest "$@" -v --timeout 120 --timeout-method thread -x > gpurun_out/$name.log 2>&1; local rc=$?; tail -25 gpurun_out/$name.log; [ $rc -ne 0 ] && { echo "$name failed rc=$rc"; exit $rc; }; return 0; }
run pcond tests/test_gpu_pcond.py
run wide tests/test_gpu_wide_ipm.py
run widegold tests/test_gpu_parity.py -k "w_ or condw or fullw"
