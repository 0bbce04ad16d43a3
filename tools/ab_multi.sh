#!/bin/bash
# alternating A/B of several engine builds on C2 (auto): bash tools/ab_multi.sh DIR1 DIR2 ...
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2 3; do
  for d in "$@"; do
    timeout -k 10 120 python tools/ab_lib.py "$d" auto 1000 || exit 1
  done
done > gpurun_out/abm.txt 2>&1
cat gpurun_out/abm.txt
