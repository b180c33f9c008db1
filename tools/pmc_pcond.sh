#!/bin/bash
# Instruction-mix counters of hk_pcond alone (tools/pcond_time.py workload), one rocprofv3 pass per counter group
# -> gpurun_out/pmc_pcond.json.  Usage: tools/pmc_pcond.sh [tag]
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out/pcmix_$tag
export TMPDIR=/tmp
run() { local d=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pcmix_$tag/$d -o run --output-format csv -- python3 tools/pcond_time.py > gpurun_out/pcmix_$tag/$d.log 2>&1 || { echo "pmc $d failed"; tail -5 gpurun_out/pcmix_$tag/$d.log; exit 1; }; echo "pass $d ok"; }
run a SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
run b SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM
python3 tools/pmc_mix_summarize.py gpurun_out/pcmix_$tag gpurun_out/pmc_pcond_$tag.json
