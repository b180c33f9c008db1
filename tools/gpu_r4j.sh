#!/bin/bash
# Round-4 evidence batch 10 (one gpurun call): VERDICT r3 item 4's same-box A/B of the load width on the stage fetches:
# hpmpc_amd/lib/ab/libW.so (HK_WIDE_BOP: the factorisation's and the corrector's BAbt operand registers 1-2 of the
# compiled (4, 12) class in one 16-B load per lane, ld_pair16) against the in-tree build (libFinal.so), after the parity
# subset on W.  Every GPU step has its own limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/libW.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_configs3.py -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/tests_W.log 2>&1 \
  || { tail -30 gpurun_out/tests_W.log; exit 1; }
echo "W $(tail -1 gpurun_out/tests_W.log)"
AB_SKIP_TESTS=1 AB_VARIANTS="Final W" bash tools/gpu_ab.sh || exit 1
