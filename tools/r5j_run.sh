# A/B: kernel events on the timed steps (--timed-events) vs on the last warmup steps
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  AB_WARMUP=60 AB_ARGS="" bash tools/ab_quick.sh r5j_def$i "cfg3 cfg2 k256"
  AB_WARMUP=60 AB_ARGS="--timed-events" bash tools/ab_quick.sh r5j_tev$i "cfg3 cfg2 k256"
done
