#!/bin/bash
# Round-4 evidence batch 8 (one gpurun call): the parity subset on hpmpc_amd/lib/ab/libO.so (O: the Riccati entry
# points' backward sweep with stage k-2 in flight, ric_backward PD = 2), then same-box A/Bs of L and O with the
# Riccati legs (N=100 sv batch, configs[2]).  Every GPU step has its own limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/libO.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_configs2.py tests/test_gpu_iface.py tests/test_gpu_pcond.py -m gpu -q --maxfail=3 --timeout 300 \
  --timeout-method thread > gpurun_out/tests_O.log 2>&1 || { tail -30 gpurun_out/tests_O.log; exit 1; }
echo "O $(tail -1 gpurun_out/tests_O.log)"
AB_SKIP_TESTS=1 AB_VARIANTS="L O" bash tools/gpu_ab.sh ric || exit 1
