#!/bin/bash
# PMC passes for bench.py's roofline record (GPU box), each counter group in
# its own rocprofv3 run (no trace domains), then the per-call summary:
#   bash tools/pmc_roofline.sh <outdir> <key> <stripes> [bench args...]
# e.g. bash tools/pmc_roofline.sh gpurun_out/pmc_cfg3 cfg3 1024 --cfg cfg3
# The record lands in <outdir>/pmc_roofline.json (copy it into
# profiles/pmc_roofline.json's "configs" with tools/pmc_roofline.py).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1
KEY=$2
S=$3
shift 3
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
    local name=$1
    shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT" -o "$name" \
        -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 $BENCH_ARGS \
        > "$OUT/$name.log" 2>&1
}
BENCH_ARGS="$*"
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
python3 "$R/tools/pmc_roofline.py" "$OUT" "$KEY" "$S" "$OUT/pmc_roofline.json"
