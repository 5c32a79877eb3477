#!/bin/bash
set -o pipefail
bash tools/prof.sh gpurun_out/s15/prof2 --steps 5 --no-cpu-baseline &&
bash tools/prof.sh gpurun_out/s15/prof3 --steps 5 --no-cpu-baseline --cfg cfg3 &&
bash tools/prof.sh gpurun_out/s15/profs --steps 5 --no-cpu-baseline --systematic
