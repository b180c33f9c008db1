#!/bin/bash
# Round-end evidence on the GPU box: GPU parity tests, smoke, the counter passes (instruction mix / stalls and the
# calibrated HBM traffic, tools/pmc_mix.sh -> profiles/pmc_hk_ipm.json before the bench reads it), the default
# bench line, and the rocprofv3 kernel stats of the same bench command.  Every GPU step has its own time limit;
# the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
R=${1:-r02}
step() { local name=$1; shift; echo "== $name"; "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -${TAILN:-3} gpurun_out/$name.log; if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; exit $rc; fi; }
step tests timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step smoke timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step pmc bash tools/pmc_mix.sh
cp gpurun_out/pmc_hk_ipm.json profiles/pmc_hk_ipm.json && cp gpurun_out/pmc_mix.json gpurun_out/${R}_pmc_mix.json
step hbmbw timeout -k 10 120 python3 tools/hbm_bw.py
grep '^{' gpurun_out/hbmbw.log | tail -1 > gpurun_out/${R}_hbm_bw.json
step bench timeout -k 10 600 python3 bench.py
grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/${R}_bench.json
# kernel stats of the timed region only: no warmup queue, no isolated batch, so every hk_ipm_* launch
# in the trace is one of the timed queue's (its average matches the bench line's launch_ms)
step stats timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats -o run --output-format csv -- python3 bench.py --no-cpu --warmup 0 --no-isolated --no-queue-batch-slots --no-aliased --no-coupled --no-k40
find gpurun_out/prof/stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${R}_kernel_stats.csv \;
head -12 gpurun_out/${R}_kernel_stats.csv | cut -c1-160
