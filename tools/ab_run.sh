# A/B only (no parity suite): bench lines of the product build against
# build/ab/<variants> over AB_CFGS (tools/ab_quick.sh)
set -e
cd $GRAFT_REPO_ROOT
AB_WARMUP=${AB_WARMUP:-60} bash tools/ab_quick.sh ${AB_TAG:-ab} "${AB_CFGS:-cfg3}" ${AB_VARIANTS:-prev}
