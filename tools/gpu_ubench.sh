#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/check_gpu.py > gpurun_out/check.log 2>&1 || { echo "check failed $?"; cat gpurun_out/check.log; exit 1; }
grep -E "^(sv|trf|ipm)" gpurun_out/check.log
timeout -k 10 300 python3 tools/ubench.py > gpurun_out/ubench.log 2>&1 || { echo "ubench failed $?"; cat gpurun_out/ubench.log; exit 1; }
cat gpurun_out/ubench.log | grep -v amdgpu.ids
