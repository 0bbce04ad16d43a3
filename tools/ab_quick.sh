#!/bin/bash
# alternating A/B of build/ab_old vs the package build on C2 (auto) and the reference's example,
# then the wave-schedule parity subset and the device-math tests
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python tools/ab_lib.py build/ab_old auto 1000 || exit 1
  timeout -k 10 120 python tools/ab_lib.py gfp_gaussian_process_amd/lib auto 1000 || exit 1
done > gpurun_out/ab.txt 2>&1
for i in 1 2; do
  timeout -k 10 120 python tools/ab_lib.py build/ab_old auto 0 || exit 1
  timeout -k 10 120 python tools/ab_lib.py gfp_gaussian_process_amd/lib auto 0 || exit 1
done >> gpurun_out/ab.txt 2>&1
cat gpurun_out/ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_math.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "device or wave or synthetic or example" > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab_pytest.log; exit $rc
