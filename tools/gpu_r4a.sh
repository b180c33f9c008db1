#!/bin/bash
# Round-4 evidence batch (one gpurun call): parity suite, quick bench line, HBM load-width probes, then same-box A/Bs of
# hpmpc_amd/lib/ab/lib{A,B,C}.so -- A: hand-over without fences (HK_MW_FENCE=0), B: the in-tree build,
# C: -ffp-contract=on, D: no clamp certificate (HK_COUNT_NOCERT, timing only), E: gain-form trs u solve, F: E + mu_aff
# accumulated in the predictor sweep -- on the lone-QP latency (A B C) and on the headline queue (B D E F).  Every GPU step has its own limit; the
# script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_quickbench.sh || exit 1
timeout -k 10 300 python3 tools/hbm_bw.py > gpurun_out/hbm_bw.json 2> gpurun_out/hbm_bw.err || { tail -5 gpurun_out/hbm_bw.err; exit 1; }
cat gpurun_out/hbm_bw.json
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/libhpmpc_mi355x_stamps.so timeout -k 10 300 python3 tools/xfac_rate.py > gpurun_out/xfac_rate.json 2> gpurun_out/xfac_rate.err || { tail -5 gpurun_out/xfac_rate.err; exit 1; }
cat gpurun_out/xfac_rate.json
AB_SKIP_TESTS=1 AB_VARIANTS="A B C" bash tools/gpu_ab.sh latency || exit 1
AB_SKIP_TESTS=1 AB_VARIANTS="B D E F" bash tools/gpu_ab.sh || exit 1
# F (mu_aff accumulated in the predictor sweep) against the oracle / goldens before it becomes the in-tree build
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/libF.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_ipm2.py tests/test_gpu_configs3.py -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread \
  > gpurun_out/tests_F.log 2>&1; tail -3 gpurun_out/tests_F.log
