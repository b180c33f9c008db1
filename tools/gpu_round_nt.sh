# Round evidence without the GPU test suite (tools/gpu_round.sh minus its first two steps): counter passes, HBM
# bandwidth probe, the default bench line and the rocprofv3 kernel stats of the timed queue.  R: the round tag.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
R=${1:-r06}
bash tools/pmc_mix.sh > gpurun_out/pmc.log 2>&1 || { tail -20 gpurun_out/pmc.log; exit 1; }
tail -30 gpurun_out/pmc.log
cp gpurun_out/pmc_hk_ipm.json profiles/pmc_hk_ipm.json && cp gpurun_out/pmc_mix.json gpurun_out/${R}_pmc_mix.json
timeout -k 10 120 python3 tools/hbm_bw.py > gpurun_out/hbmbw.log 2>&1 && grep '^{' gpurun_out/hbmbw.log | tail -1 > gpurun_out/${R}_hbm_bw.json
timeout -k 10 600 python3 bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/${R}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats -o run --output-format csv -- python3 bench.py --no-cpu --warmup 0 --no-isolated --no-queue-batch-slots --no-aliased --no-coupled --no-k40 > gpurun_out/stats.log 2>&1 || { tail -20 gpurun_out/stats.log; exit 1; }
find gpurun_out/prof/stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${R}_kernel_stats.csv \;
cp profiles/pmc_hk_ipm.json gpurun_out/${R}_pmc_hk_ipm.json
head -12 gpurun_out/${R}_kernel_stats.csv | cut -c1-160
