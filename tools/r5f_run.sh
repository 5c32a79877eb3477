# k > 128 context rework: GPU parity suite, context stage probe, A/B
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5f
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5f/gpu.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r5f/gpu.log | tail -40; exit 1; }
tail -1 gpurun_out/r5f/gpu.log
QI_LIB_PATH=build/ab/ctxbig_ts/libquadiron_amd.so timeout -k 10 200 python3 tools/ctxbig_stages.py 300,212,32,32768 256,768,256,2048 200,56,64,32768 384,128,32,32768
AB_WARMUP=${AB_WARMUP:-60} bash tools/ab_quick.sh ${AB_TAG:-r5f} "${AB_CFGS:-k300 k384 k200 k256}" prev
