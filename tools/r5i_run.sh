# parity suite, then the overlapped-context A/B (bench --ctx-stream 1 / 0)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5i
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5i/gpu.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r5i/gpu.log | tail -40; exit 1; }
tail -1 gpurun_out/r5i/gpu.log
for i in 1 2; do
  AB_WARMUP=60 AB_ARGS="--ctx-stream 1" bash tools/ab_quick.sh r5i_on$i "cfg3 cfg2 cfg3:sys k32"
  AB_WARMUP=60 AB_ARGS="--ctx-stream 0" bash tools/ab_quick.sh r5i_off$i "cfg3 cfg2 cfg3:sys k32"
done
