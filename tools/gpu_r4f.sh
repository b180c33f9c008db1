#!/bin/bash
# Round-4 evidence batch 6 (one gpurun call): the parity subset on hpmpc_amd/lib/ab/libM.so (M: the multi-wave
# kernel's sweeps as out-of-line functions, HK_MW_NOINLINE -- the register allocator then sees one sweep's roles at a
# time: SGPR-spill lane ops 4 381 -> ~900 in the kernel plus 4-240 per sweep function), then same-box A/Bs of L and M
# on the lone-QP latency and the headline queue.  Every GPU step has its own limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/libM.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_ipm2.py tests/test_gpu_configs3.py tests/test_gpu_iface.py -m gpu -q --maxfail=3 --timeout 300 \
  --timeout-method thread > gpurun_out/tests_M.log 2>&1 || { tail -30 gpurun_out/tests_M.log; exit 1; }
echo "M $(tail -1 gpurun_out/tests_M.log)"
AB_SKIP_TESTS=1 AB_VARIANTS="L M" bash tools/gpu_ab.sh latency || exit 1
AB_SKIP_TESTS=1 AB_VARIANTS="L M" bash tools/gpu_ab.sh || exit 1
