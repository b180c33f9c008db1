#!/bin/bash
# One gpurun call = a sequence of GPU steps, each under its own time limit, stopping at the first failure (no GPU step
# runs after a fault, an abort or a timeout).  Replaces the one-off round-4 batch scripts (gpu_r4*.sh).
#   tools/gpu_steps.sh "name|seconds|command" ...
# Step <name> writes gpurun_out/<name>.log; its last $TAIL (15) lines are printed.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name (${secs} s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n "${TAIL:-15}"
  if [ $rc -ne 0 ]; then
    echo "== $name failed ($rc)"
    exit $rc
  fi
done
