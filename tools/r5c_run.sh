# round-5 A/B pass: GPU parity suite, context-kernel times, cfg3 A/B against
# build/ab/prev (tools/ab_build.sh)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5c
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5c/gpu.log 2>&1
tail -3 gpurun_out/r5c/gpu.log
for v in main prev main prev; do
  L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
  echo "== $v"; QI_LIB_PATH=$L timeout -k 10 120 python3 tools/ctx_time.py 64,960,1024,2048 32,96,2048,16384 16,48,4096,32768
done
AB_WARMUP=60 bash tools/ab_quick.sh ${AB_TAG:-r5c} "${AB_CFGS:-cfg3}" prev
