#!/bin/bash
# one summary line per bench log:  bash tools/lines.sh gpurun_out/<tag>
for f in "$1"/bench*.log; do
  printf "%-28s " "$(basename $f)"
  grep -o '"value": [0-9.]*\|"encode_kernel_ms": [0-9.]*\|"decode_ms": [0-9.]*\|roundtrip_ok": [a-z]*' "$f" | tr '\n' ' '
  echo
done
