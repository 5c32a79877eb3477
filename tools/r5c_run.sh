# round-5 A/B pass: GPU parity suite, then bench lines of the product build
# against build/ab/<variants> (tools/ab_build.sh) over AB_CFGS
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5c
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5c/gpu.log 2>&1
tail -3 gpurun_out/r5c/gpu.log
AB_WARMUP=${AB_WARMUP:-60} bash tools/ab_quick.sh ${AB_TAG:-r5c} "${AB_CFGS:-cfg3}" ${AB_VARIANTS:-prev}
