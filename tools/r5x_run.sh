# A/B of a context-kernel variant: ctx_time + cfg3 bench lines
set -e
cd $GRAFT_REPO_ROOT
for v in main ${AB_VARIANTS:-n128} main ${AB_VARIANTS:-n128}; do
  L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
  echo "== $v"; QI_LIB_PATH=$L timeout -k 10 120 python3 tools/ctx_time.py 64,960,1024,2048 48,80,1024,2048
done
AB_WARMUP=60 bash tools/ab_quick.sh ${AB_TAG:-r5x} "cfg3" ${AB_VARIANTS:-n128}
