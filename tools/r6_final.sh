#!/bin/bash
# Round-6 measurement pass (GPU box), in two calls:
#   bash tools/r6_final.sh <tag> main   GPU parity suite, smoke, every bench
#                                       line, rocprofv3 kernel stats, host rate
#   (or the same in two calls: main1 = suite, smoke, bench lines;
#    main2 = rocprofv3 kernel stats, host rate)
#   bash tools/r6_final.sh <tag> pmc    the PMC roofline record of every bench
#                                       configuration (profiles/pmc_roofline.json)
# Bench lines other than the driver's default run take 30 warmup steps (60
# at cfg3 / cfg3p64 / cfg1, whose steps are ~1 ms): the GPU clock settles
# over the first tens of ms of load (tools/ramp.py).
set -o pipefail
T=${1:-r6}; PART=${2:-main}
O=gpurun_out/$T
mkdir -p $O
line() {  # cfg label -> short summary of the bench line
  python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), 'ctx', round(d['decode_ctx_ms'],4), d['roundtrip_ok'])"
}
wu() { case $1 in cfg3|cfg3p64|cfg1) echo 60;; *) echo 30;; esac; }
if [ "$PART" = main ] || [ "$PART" = main1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit $?
  timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 || exit $?
  line $O/bench.log cfg2
  timeout -k 10 300 python3 bench.py --systematic --no-cpu-baseline --warmup 30 > $O/bench_sys.log 2>&1 || exit $?
  line $O/bench_sys.log cfg2_sys
  for c in cfg3 cfg1 k32 k128 k200 k256 k300 k384 k1000 k600 cfg3p64; do
    timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline --warmup $(wu $c) > $O/bench_$c.log 2>&1 || exit $?
    line $O/bench_$c.log $c
  done
  timeout -k 10 300 python3 bench.py --cfg cfg3 --systematic --no-cpu-baseline --warmup 60 > $O/bench_cfg3_sys.log 2>&1 || exit $?
  line $O/bench_cfg3_sys.log cfg3_sys
  for c in k200 k300 k384 k600; do
    timeout -k 10 300 python3 bench.py --cfg $c --systematic --no-cpu-baseline --warmup 30 > $O/bench_${c}_sys.log 2>&1 || exit $?
    line $O/bench_${c}_sys.log ${c}_sys
  done
fi
if [ "$PART" = main ] || [ "$PART" = main2 ]; then
  for c in cfg2 cfg3 k200 k256 k300 k384 k1000 k600; do
    bash tools/prof.sh $O/prof_$c --cfg $c --steps 10 --warmup $(wu $c) --no-cpu-baseline --no-secondary || exit $?
  done
  bash tools/prof.sh $O/prof_k600_sys --cfg k600 --systematic --steps 10 --warmup 30 --no-cpu-baseline --no-secondary || exit $?
  timeout -k 10 400 python3 tools/host_rate.py > $O/host_rate.json 2> $O/host_rate.err || exit $?
fi
if [ "$PART" = pmc ]; then
  bash tools/pmc_roofline.sh $O/pmc_cfg2 cfg2 4096 --no-secondary || exit $?
  bash tools/pmc_roofline.sh $O/pmc_sys cfg2_sys 4096 --systematic || exit $?
  for c in "cfg3 1024" "cfg1 100" "k32 1024" "k128 128" "k200 64" "k256 256" "k300 32" "k384 32" "k1000 16" "k600 16" "cfg3p64 64"; do
    set -- $c
    bash tools/pmc_roofline.sh $O/pmc_$1 $1 $2 --cfg $1 --no-secondary || exit $?
  done
  for c in "cfg3 1024" "k300 32" "k600 16"; do
    set -- $c
    bash tools/pmc_roofline.sh $O/pmc_$1_sys $1_sys $2 --cfg $1 --systematic --no-secondary || exit $?
  done
fi
