#!/bin/bash
# Round-4 evidence batch 7 (one gpurun call): the parity subset on hpmpc_amd/lib/ab/libN.so (N: the multi-wave
# kernel's sweeps as out-of-line functions, HK_MW_NOINLINE, with their pointers re-made wave-uniform and the stage
# tables re-made LDS at entry (mw_uni); batch 6's M without that ran every buffer access in a waterfall loop), then same-box A/Bs of L and N
# on the lone-QP latency.  Every GPU step has its own limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/libN.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_ipm2.py tests/test_gpu_configs3.py tests/test_gpu_iface.py -m gpu -q --maxfail=3 --timeout 300 \
  --timeout-method thread > gpurun_out/tests_N.log 2>&1 || { tail -30 gpurun_out/tests_N.log; exit 1; }
echo "N $(tail -1 gpurun_out/tests_N.log)"
AB_SKIP_TESTS=1 AB_VARIANTS="L N" bash tools/gpu_ab.sh latency || exit 1
