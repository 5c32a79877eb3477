#!/bin/bash
set -o pipefail
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s16_pytest.log 2>&1 &&
bash tools/gpu_s15.sh
