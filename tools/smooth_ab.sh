#!/bin/bash
# alternate the package's engine and tools/ab_ou/ (a variant build: build_ext's engine line into
# tools/ab_ou/libggp.so, with a copy of lib/libggp_host.so) under tools/smooth_ab.py
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  for lib in gfp_gaussian_process_amd/lib tools/ab_ou; do
    for t in ${TREES:-125000}; do timeout -k 10 200 python tools/smooth_ab.py $lib $t || exit 1; done
  done
done > gpurun_out/smooth_ab.txt 2>&1
cat gpurun_out/smooth_ab.txt
