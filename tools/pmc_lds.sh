#!/bin/bash
# One SQ PMC pass (issue, waits, LDS bank conflicts) over a bench config:
#   bash tools/pmc_lds.sh <outdir> [bench args...]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1
shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE \
    --output-format csv -d "$OUT" -o sq \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 2 --warmup 1 "$@" > "$OUT/sq.log" 2>&1
