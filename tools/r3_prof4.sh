#!/bin/bash
# rocprofv3 kernel stats of several bench configs (GPU box)
#   bash tools/r3_prof4.sh <tag> <cfg>...
set -o pipefail
T=$1; shift
for c in "$@"; do
  bash tools/prof.sh gpurun_out/$T/$c --cfg $c --steps 10 --no-cpu-baseline || exit $?
done
