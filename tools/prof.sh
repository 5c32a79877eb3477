#!/bin/bash
# rocprofv3 kernel-trace + stats of a bench run (GPU box).  Usage:
#   bash tools/prof.sh <outdir> [bench args...]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1
shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
    -- python3 "$R/bench.py" "$@" > "$OUT/bench.log" 2>&1
