#!/bin/bash
# lane kernel with the OU constants in scalar registers (-DPROBE_SOU: ab_sou) and that at two
# waves per SIMD (ab_sou2), against the shipped engine (ab_new): C5 shard (tools/lane_ab_c5.py)
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  for b in new sou sou2; do timeout -k 10 200 python tools/lane_ab_c5.py build/ab_$b || exit 1; done
done > gpurun_out/r4i.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r4i.txt; exit $rc
