#!/bin/bash
# Instruction-mix / stall counters of the IPM pass kernels on the benchmark queue (diagnostic).
set -o pipefail
mkdir -p gpurun_out/mix
export TMPDIR=/tmp
run() { timeout -k 10 300 rocprofv3 --pmc "$@" -d gpurun_out/mix/$1 -o run --output-format csv -- python3 tools/pmc_run.py > gpurun_out/mix/$1.log 2>&1 || { echo "pmc $1 failed"; tail -5 gpurun_out/mix/$1.log; exit 1; }; }
run SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY
run SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA
run SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM
run SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64
echo done
