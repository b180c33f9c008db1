#!/bin/bash
# Round-4 evidence batch 4 (one gpurun call): the parity subset on hpmpc_amd/lib/ab/libK.so (K: the factorisation's
# stage loop instantiated twice, forming the certificate bounds in a solve's first factorisation and loading them in
# the others, instead of one loop with a run-time branch), same-box A/Bs of I and K, and the certificate failure
# counts per stage and per backward sweep (stamps build).  Every GPU step has its own limit; the script stops at the
# first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/libK.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_ipm2.py tests/test_gpu_configs3.py -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread \
  > gpurun_out/tests_K.log 2>&1 || { tail -30 gpurun_out/tests_K.log; exit 1; }
echo "K $(tail -1 gpurun_out/tests_K.log)"
AB_SKIP_TESTS=1 AB_VARIANTS="I K" bash tools/gpu_ab.sh || exit 1
AB_SKIP_TESTS=1 AB_VARIANTS="I K" bash tools/gpu_ab.sh latency || exit 1
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/libhpmpc_mi355x_stamps.so timeout -k 10 300 python3 tools/xfac_rate.py > gpurun_out/xfac_rate.json 2> gpurun_out/xfac_rate.err || { tail -5 gpurun_out/xfac_rate.err; exit 1; }
cat gpurun_out/xfac_rate.json
