# parity suite, then A/B of the KS >= 8 operand-stationary geometry, then a
# PMC read/write pass of the product build at k200 / k256 / k300 / k384 / k128
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5k
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5k/gpu.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r5k/gpu.log | tail -40; exit 1; }
tail -1 gpurun_out/r5k/gpu.log
AB_WARMUP=30 bash tools/ab_quick.sh r5k "k200 k256 k300 k384 k128 k300:sys" prev ks8
for c in k200:64 k256:256 k300:32 k128:128; do
  k=${c%:*}; S=${c#*:}
  bash tools/pmc_roofline.sh gpurun_out/r5k/pmc_$k $k $S --cfg $k --no-secondary > /dev/null
done
