#!/bin/bash
# occupancy probe (diagnostic): the lane kernels with the outputs stage stubbed out (values
# meaningless) at the default register budget (ab_stub1) and at two waves per SIMD (ab_stub2),
# against the shipped engine (ab_new) on a C5 shard: what a two-wave lane step could gain
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  for b in new stub1 stub2; do timeout -k 10 200 python tools/lane_ab_c5.py build/ab_$b || exit 1; done
done > gpurun_out/lane_ab_r4g.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/lane_ab_r4g.txt; exit $rc
