#!/bin/bash
# alternating A/B of build/ab_old vs build/ab_new on C2 (auto) and the reference's example
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python tools/ab_lib.py build/ab_old auto 1000 || exit 1
  timeout -k 10 120 python tools/ab_lib.py build/ab_new auto 1000 || exit 1
  timeout -k 10 120 python tools/ab_lib.py build/ab_old auto 0 || exit 1
  timeout -k 10 120 python tools/ab_lib.py build/ab_new auto 0 || exit 1
done > gpurun_out/wave_ab.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/wave_ab.txt; exit $rc
