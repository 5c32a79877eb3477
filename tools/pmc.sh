#!/bin/bash
# PMC passes over a short bench run (each pass its own rocprofv3 run: the
# TCC FETCH_SIZE / WRITE_SIZE counters do not fit one pass).  Usage on the GPU
# box:   bash tools/pmc.sh <outdir> [bench args...]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1
shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
    local name=$1
    shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT" -o "$name" \
        -- python3 "$R/bench.py" --no-cpu-baseline $BENCH_ARGS > "$OUT/$name.log" 2>&1
}
BENCH_ARGS="$*"
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit $?
run sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_INSTS_LDS || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
echo done
