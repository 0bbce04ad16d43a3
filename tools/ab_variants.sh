#!/bin/bash
# alternating A/B of engine builds on C2 (auto, 1000 trees) and the reference's example, each run
# after 300 ms of full-chip work (the sustained clock): tools/ab_variants.sh LIB_DIR [LIB_DIR ...]
set -o pipefail
export TMPDIR=/tmp AB_PREHEAT_MS=300; mkdir -p gpurun_out
for i in 1 2 3; do
  for d in "$@"; do timeout -k 10 120 python tools/ab_lib.py $d auto 1000 || exit 1; done
done > gpurun_out/ab_variants.txt 2>&1
for i in 1 2; do
  for d in "$@"; do timeout -k 10 120 python tools/ab_lib.py $d auto 0 || exit 1; done
done >> gpurun_out/ab_variants.txt 2>&1
grep ms/eval gpurun_out/ab_variants.txt
