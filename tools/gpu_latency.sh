# lone-QP latency probe (tools/latency_probe.py), after the GPU parity suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
tail -3 gpurun_out/tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 tools/latency_probe.py > gpurun_out/latency.log 2>&1 || { tail -20 gpurun_out/latency.log; exit 1; }
grep -v amdgpu.ids gpurun_out/latency.log
