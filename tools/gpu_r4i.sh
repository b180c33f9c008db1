#!/bin/bash
# Round-4 evidence batch 9 (one gpurun call): parity subsets on hpmpc_amd/lib/ab/lib{O,P}.so -- O: the Riccati entry
# points' backward sweep with stage k-2 in flight (ric_backward PD = 2); P: O with the update pass loading six
# stages per chunk instead of four (HK_UPD_CH=6); R: O with the multi-wave tile wave's certificate ballot taken after
# the u blocks (CertDefer) -- then same-box A/Bs: L vs O with the Riccati legs (N=100 sv batch, configs[2]), O vs P on
# the headline queue, O vs R on the lone-QP latency.  Every GPU step has its own limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in O P R; do
  HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/lib$v.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_configs2.py tests/test_gpu_configs3.py tests/test_gpu_iface.py -m gpu -q --maxfail=3 --timeout 300 \
    --timeout-method thread > gpurun_out/tests_$v.log 2>&1 || { tail -30 gpurun_out/tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/tests_$v.log)"
done
AB_SKIP_TESTS=1 AB_VARIANTS="L O" bash tools/gpu_ab.sh ric || exit 1
AB_SKIP_TESTS=1 AB_VARIANTS="O P" bash tools/gpu_ab.sh || exit 1
AB_SKIP_TESTS=1 AB_VARIANTS="O R" bash tools/gpu_ab.sh latency || exit 1
