#!/bin/bash
# A/B of the engine built with -ffp-contract=fast (build/ab_new) against HEAD's (build/ab_old):
# lane-schedule legs, C2 and the example; values printed for the parity record
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python tools/lane_ab.py build/ab_old || exit 1
  timeout -k 10 200 python tools/lane_ab.py build/ab_new || exit 1
  timeout -k 10 120 python tools/ab_lib.py build/ab_old auto 1000 || exit 1
  timeout -k 10 120 python tools/ab_lib.py build/ab_new auto 1000 || exit 1
  timeout -k 10 120 python tools/ab_lib.py build/ab_old auto 0 || exit 1
  timeout -k 10 120 python tools/ab_lib.py build/ab_new auto 0 || exit 1
done > gpurun_out/fma_ab.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/fma_ab.txt; exit $rc
