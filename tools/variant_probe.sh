#!/bin/bash
# Build a kernel variant on the GPU box (HK_EXTRA_FLAGS) and run the queue probe on it (diagnostic).
set -o pipefail
export PYTHONPATH=.
for V in "$@"; do
  echo "== variant: $V"
  HK_EXTRA_FLAGS="$V" timeout -k 10 300 python3 -c "from hpmpc_amd.build import build_hip; build_hip(force=True)" > gpurun_out/vbuild.log 2>&1 || { tail -5 gpurun_out/vbuild.log; exit 1; }
  QP_SLOTS="${QP_SLOTS:-2048 3072}" timeout -k 10 300 python3 tools/queue_probe.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done
