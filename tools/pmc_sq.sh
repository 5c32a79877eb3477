#!/bin/bash
# One SQ PMC pass (instruction mix, waits, issue) over any program:
#   bash tools/pmc_sq.sh <outdir> <program> [args...]
# e.g. bash tools/pmc_sq.sh gpurun_out/x/sq_bench python3 bench.py --cfg cfg3 --steps 2 --warmup 1 --no-cpu-baseline
#      bash tools/pmc_sq.sh gpurun_out/x/sq_probe ./build/membw7
# Summary: python3 tools/pmc_sq_summary.py <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1
shift
mkdir -p "$OUT"
# relative paths (the program, bench.py) against the repo root: rocprofv3
# runs from /tmp
ARGS=()
for a in "$@"; do
  case "$a" in /*|-*) ARGS+=("$a") ;; *) if [ -e "$R/$a" ]; then ARGS+=("$R/$a"); else ARGS+=("$a"); fi ;; esac
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT" -o sq -- "${ARGS[@]}" > "$OUT/sq.log" 2>&1
