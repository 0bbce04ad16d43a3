#!/bin/bash
# alternating A/B of the package build against build/ab_new on C2 (auto, 1000 trees) and the
# reference's example, each run after 300 ms of full-chip work (the sustained clock)
set -o pipefail
export TMPDIR=/tmp AB_PREHEAT_MS=300; mkdir -p gpurun_out
for i in 1 2 3; do
  for d in gfp_gaussian_process_amd/lib build/ab_new; do timeout -k 10 120 python tools/ab_lib.py $d auto 1000 || exit 1; done
done > gpurun_out/ab_c2.txt 2>&1
for i in 1 2; do
  for d in gfp_gaussian_process_amd/lib build/ab_new; do timeout -k 10 120 python tools/ab_lib.py $d auto 0 || exit 1; done
done >> gpurun_out/ab_c2.txt 2>&1
grep ms/eval gpurun_out/ab_c2.txt
