#!/bin/bash
# Round-4 evidence batch 2 (one gpurun call): parity suite + quick bench line on the in-tree build (H: gain-form trs,
# pi formed at the next stage, 256-B workspace slots, unfenced hand-over), same-box A/Bs of hpmpc_amd/lib/ab/lib{E,H}.so
# on the headline queue and of lib{A,E,H}.so on the lone-QP latency, then the multi-wave kernel's per-body cycles
# (stamps build).  Every GPU step has its own limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_quickbench.sh || exit 1
AB_SKIP_TESTS=1 AB_VARIANTS="E H" bash tools/gpu_ab.sh || exit 1
AB_SKIP_TESTS=1 AB_VARIANTS="A E H" bash tools/gpu_ab.sh latency || exit 1
HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/libhpmpc_mi355x_stamps.so timeout -k 10 300 python3 tools/mw_phases.py \
  > gpurun_out/mw_phases.txt 2>&1 || { tail -5 gpurun_out/mw_phases.txt; exit 1; }
cat gpurun_out/mw_phases.txt
