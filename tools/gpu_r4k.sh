#!/bin/bash
# Round-4 evidence batch 11 (one gpurun call): hpmpc_amd/lib/ab/libX.so (X: the clamped fallback branch of
# stage_chol marked cold, HK_XFAC_UNLIKELY) against the in-tree build (libBase.so): parity subset on X, then same-box
# A/Bs on the lone-QP latency and the headline queue.  Every GPU step has its own limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/libX.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_configs3.py -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/tests_X.log 2>&1 \
  || { tail -30 gpurun_out/tests_X.log; exit 1; }
echo "X $(tail -1 gpurun_out/tests_X.log)"
AB_SKIP_TESTS=1 AB_VARIANTS="Base X" bash tools/gpu_ab.sh latency || exit 1
AB_SKIP_TESTS=1 AB_VARIANTS="Base X" bash tools/gpu_ab.sh || exit 1
