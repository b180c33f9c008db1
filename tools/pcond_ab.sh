set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do for v in ${AB_VARIANTS:-P1 P2}; do
  HPMPC_MI355X_LIB=$PWD/hpmpc_amd/lib/ab/lib$v.so timeout -k 10 120 python3 tools/pcond_time.py > gpurun_out/pab_$v$i.log 2>&1 || exit 1
  echo "$v$i $(cat gpurun_out/pab_$v$i.log | tr '\n' ' ')"
done; done
