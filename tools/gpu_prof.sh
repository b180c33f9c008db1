#!/bin/bash
# per-kernel time breakdown of the benchmark workload (rocprofv3 kernel trace)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/kprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/kprof.log 2>&1 || { echo "prof failed $?"; tail -20 gpurun_out/kprof.log; exit 1; }
tail -1 gpurun_out/kprof.log | cut -c1-400
f=$(find gpurun_out/kprof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print(f"{r['Name'][:40]:40s} calls {int(r['Calls']):5d}  total {float(r['TotalDurationNs'])/1e6:9.3f} ms  avg {float(r['AverageNs'])/1e3:9.1f} us  {float(r['Percentage']):5.1f}%")
PY
