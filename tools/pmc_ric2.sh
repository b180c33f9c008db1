#!/bin/bash
# Instruction-mix / stall counters of the one-wave (hk_ric_sv) and two-wave (hk_ric_sv2) Riccati sv kernels at the
# benchmark batch (tools/ric_pmc_run.py), one rocprofv3 pass per counter group -> gpurun_out/pmc_ric2.json.
set -o pipefail
mkdir -p gpurun_out/ric2mix
export TMPDIR=/tmp
run() { local d=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/ric2mix/$d -o run --output-format csv -- python3 tools/ric_pmc_run.py > gpurun_out/ric2mix/$d.log 2>&1 || { echo "pmc $d failed"; tail -5 gpurun_out/ric2mix/$d.log; exit 1; }; echo "pass $d ok"; }
run a SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
run b SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS
run c SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
python3 tools/pmc_mix_summarize.py gpurun_out/ric2mix gpurun_out/pmc_ric2.json
