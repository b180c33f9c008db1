#!/bin/bash
# Instruction-mix / stall counters (one rocprofv3 pass per counter group), then the calibrated HBM traffic
# (FETCH_SIZE / WRITE_SIZE passes) of the IPM pass kernels, the Riccati sv and the configs[4] pipeline, over
# tools/pmc_run.py.  Summaries: gpurun_out/pmc_mix.json, gpurun_out/pmc_hk_ipm.json.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/mix gpurun_out/prof
export TMPDIR=/tmp
run() { local d=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/mix/$d -o run --output-format csv -- python3 tools/pmc_run.py > gpurun_out/mix/$d.log 2>&1 || { echo "pmc $d failed"; tail -5 gpurun_out/mix/$d.log; exit 1; }; echo "pass $d ok"; }
run a SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
run b SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS
run c SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run d SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64
run e TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum GRBM_GUI_ACTIVE
python3 tools/pmc_mix_summarize.py gpurun_out/mix gpurun_out/pmc_mix.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run --output-format csv -- python3 tools/pmc_run.py > gpurun_out/pmc_fetch.log 2>&1 || { echo fetch failed; tail -5 gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run --output-format csv -- python3 tools/pmc_run.py > gpurun_out/pmc_write.log 2>&1 || { echo write failed; tail -5 gpurun_out/pmc_write.log; exit 1; }
KK=$(grep kk_pass gpurun_out/pmc_write.log | awk '{print $2}')
python3 tools/pmc_summarize.py gpurun_out/prof/fetch gpurun_out/prof/write gpurun_out/pmc_hk_ipm.json $KK
