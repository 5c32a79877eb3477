#!/bin/bash
# Chunked multi-stream step (encode of one slice beside the decode of another)
# vs the single-stream step, cfg2 and cfg3 (GPU box).
set -o pipefail
O=gpurun_out/chunks
mkdir -p $O
for i in 1 2; do
  for c in 1 2 4 8; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --chunks $c --streams 2 > $O/cfg2_c${c}_$i.log 2>&1 &&
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --cfg cfg3 --chunks $c --streams 2 > $O/cfg3_c${c}_$i.log 2>&1 || exit $?
  done
done
