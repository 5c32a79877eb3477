set -o pipefail
mkdir -p gpurun_out/ctx
for v in main g4; do
  L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
  QI_LIB_PATH=$L timeout -k 10 120 python3 tools/ctx_time.py > gpurun_out/ctx/$v.log 2>&1 || exit $?
done
