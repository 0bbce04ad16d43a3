#!/bin/bash
# alternating A/B of build/ab_old vs the package build (C2 auto x3, C4-shard lane x2), then
# the GPU parity suite
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python tools/ab_lib.py build/ab_old auto 1000 || exit 1
  timeout -k 10 120 python tools/ab_lib.py gfp_gaussian_process_amd/lib auto 1000 || exit 1
done > gpurun_out/ab.txt 2>&1
for i in 1 2; do
  timeout -k 10 120 python tools/ab_lib.py build/ab_old lane 12500 || exit 1
  timeout -k 10 120 python tools/ab_lib.py gfp_gaussian_process_amd/lib lane 12500 || exit 1
  timeout -k 10 120 python tools/ab_lib.py build/ab_old group 2000 || exit 1
  timeout -k 10 120 python tools/ab_lib.py gfp_gaussian_process_amd/lib group 2000 || exit 1
done >> gpurun_out/ab.txt 2>&1
cat gpurun_out/ab.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; exit $rc
