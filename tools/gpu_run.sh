#!/bin/bash
# helper executed on the GPU box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/check_gpu.py > gpurun_out/check.log 2>&1
echo "exit $?" >> gpurun_out/check.log
