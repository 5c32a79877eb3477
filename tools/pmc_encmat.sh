#!/bin/bash
# PMC passes for the encode A/B (FNT codelets vs matrix-core encode).
set -o pipefail
bash tools/pmc.sh gpurun_out/pmc_fnt_cfg3 --cfg cfg3 --steps 3 --warmup 1 &&
QI_ENC_MATRIX=1 bash tools/pmc.sh gpurun_out/pmc_mat_cfg3 --cfg cfg3 --steps 3 --warmup 1 &&
QI_ENC_MATRIX=1 bash tools/pmc.sh gpurun_out/pmc_mat_cfg2 --steps 3 --warmup 1
