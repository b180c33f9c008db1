set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh && timeout -k 10 600 python3 bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log; exit $rc
