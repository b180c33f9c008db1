#!/bin/bash
# Round-4 evidence batch 3 (one gpurun call): the parity subset (drop-in, batched and solo IPM, clamp, gates, goldens,
# alternate IPM, configs[3], reference drivers) on hpmpc_amd/lib/ab/lib{I,J}.so -- I: the clamp certificate's bounds
# formed in each solve's first factorisation instead of a per-solve pass in init / refill; J: I with the clamped
# fallback out of line (HK_FALLBACK_CALL) -- then same-box A/Bs of H, I, J on the headline queue and the lone QP.
# Every GPU step has its own limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in I J; do
  HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/lib$v.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_ipm2.py tests/test_gpu_configs3.py -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/tests_$v.log 2>&1 || { tail -30 gpurun_out/tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/tests_$v.log)"
done
AB_SKIP_TESTS=1 AB_VARIANTS="H I J" bash tools/gpu_ab.sh || exit 1
AB_SKIP_TESTS=1 AB_VARIANTS="H I J" bash tools/gpu_ab.sh latency || exit 1
