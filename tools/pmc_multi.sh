set -e
cd $GRAFT_REPO_ROOT
for c in k200:64 k300:32 k384:32 k256:256; do
  k=${c%:*}; S=${c#*:}
  bash tools/pmc_roofline.sh gpurun_out/pmc5_$k $k $S --cfg $k --no-secondary
done
