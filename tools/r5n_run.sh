# parity suite, context timing (k <= 64 A(x) split) and A/B against HEAD
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5n
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5n/gpu.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r5n/gpu.log | tail -40; exit 1; }
tail -1 gpurun_out/r5n/gpu.log
for v in main prev main prev; do
  L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
  echo "== $v"; QI_LIB_PATH=$L timeout -k 10 120 python3 tools/ctx_time.py 64,960,1024,2048 48,80,1024,2048
done
AB_WARMUP=60 bash tools/ab_quick.sh r5n "cfg3 k384 cfg3:sys" prev
