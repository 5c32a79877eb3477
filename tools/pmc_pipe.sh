#!/bin/bash
# Pipe-level PMC passes (VALU / MFMA / LDS / wait shares) over a short bench
# run, one rocprofv3 run per pass (GPU box):
#   bash tools/pmc_pipe.sh <outdir> [bench args...]     (env passes through)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1
shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
    local name=$1
    shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT" -o "$name" \
        -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 $BENCH_ARGS > "$OUT/$name.log" 2>&1
}
BENCH_ARGS="$*"
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY || exit $?
run p2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE || exit $?
run p3 SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR || exit $?
echo done
