#!/bin/bash
# alternating A/B of engine builds for one schedule and forest size:
# bash tools/ab_multi_k.sh KERNEL TREES DIR1 DIR2 ...
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
k=$1; n=$2; shift 2
for i in 1 2 3; do
  for d in "$@"; do
    timeout -k 10 120 python tools/ab_lib.py "$d" "$k" "$n" || exit 1
  done
done > gpurun_out/abk_${k}_${n}.txt 2>&1
cat gpurun_out/abk_${k}_${n}.txt
