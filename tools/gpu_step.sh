#!/bin/bash
# run on the GPU box: parity diag, smoke, bench (+ optional rocprof kernel trace)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/check_gpu.py > gpurun_out/check.log 2>&1 || { echo "check failed $?"; cat gpurun_out/check.log; exit 1; }
grep -E "^(sv|trf|ipm)" gpurun_out/check.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed $?"; cat gpurun_out/smoke.log; exit 1; }
grep smoke gpurun_out/smoke.log
timeout -k 10 400 python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench.log 2>&1 || { echo "bench failed $?"; cat gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ "$1" == "prof" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1 || { echo "prof failed $?"; tail -20 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*kernel_stats*" | head -3
  cat $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
fi
