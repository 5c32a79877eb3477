#!/bin/bash
# A/B: register FNT encode vs matrix-core encode (QI_ENC_MATRIX=1) on the
# GPU box; parity tests under the forced matrix path first.
set -o pipefail
O=gpurun_out/${1:-encmat}
mkdir -p $O
QI_ENC_MATRIX=1 timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_mat.log 2>&1 &&
for c in cfg3 cfg2; do
  timeout -k 10 200 python3 bench.py --cfg $c --no-cpu-baseline > $O/fnt_$c.log 2>&1 &&
  QI_ENC_MATRIX=1 timeout -k 10 200 python3 bench.py --cfg $c --no-cpu-baseline > $O/mat_$c.log 2>&1 || exit $?
done
