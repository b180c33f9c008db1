#!/bin/bash
# Round-4 evidence batch 5 (one gpurun call): the parity subset on hpmpc_amd/lib/ab/libL.so (L: the certificate test
# in threshold form -- T = g^2 / (1e-11 g + 1e-15) stored per stage, the diagonal from 0/1 weights instead of lane
# masks -- in the factorisations and the multi-wave tile wave), same-box A/Bs of K and L, and the certificate failure
# counts (stamps build).  Every GPU step has its own limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/libL.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_ipm2.py tests/test_gpu_configs3.py -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread \
  > gpurun_out/tests_L.log 2>&1 || { tail -30 gpurun_out/tests_L.log; exit 1; }
echo "L $(tail -1 gpurun_out/tests_L.log)"
AB_SKIP_TESTS=1 AB_VARIANTS="K L" bash tools/gpu_ab.sh || exit 1
AB_SKIP_TESTS=1 AB_VARIANTS="K L" bash tools/gpu_ab.sh latency || exit 1
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/libhpmpc_mi355x_stamps.so timeout -k 10 300 python3 tools/xfac_rate.py > gpurun_out/xfac_rate.json 2> gpurun_out/xfac_rate.err || { tail -5 gpurun_out/xfac_rate.err; exit 1; }
cat gpurun_out/xfac_rate.json
