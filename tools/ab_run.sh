#!/bin/bash
# A/B of engine variants built by tools/ab_build.sh (diagnostic): tools/ab_run.sh NAME [NAME ...]
# per-stage stamps (cycles per steady C2 step) and C2 / example ms per evaluation, alternating
set -o pipefail
export TMPDIR=/tmp AB_PREHEAT_MS=300; mkdir -p gpurun_out
OUT=gpurun_out/ab_run.txt
: > $OUT
for i in 1 2; do
  for n in "$@"; do
    echo "== stamps $n" >> $OUT
    timeout -k 10 120 build/diag/stamp_$n 1000 3 2>&1 | head -14 >> $OUT || exit 1
  done
done
for i in 1 2 3; do
  for n in "$@"; do timeout -k 10 120 python tools/ab_lib.py build/ab_$n auto 1000 2>&1 | grep ms/eval >> $OUT || exit 1; done
done
for i in 1 2; do
  for n in "$@"; do timeout -k 10 120 python tools/ab_lib.py build/ab_$n auto 0 2>&1 | grep ms/eval >> $OUT || exit 1; done
done
grep -E "==|cycles/step|ms/eval" $OUT
