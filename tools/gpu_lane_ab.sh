#!/bin/bash
# alternating A/B of build/ab_old vs build/ab_new on the lane-schedule legs (tools/lane_ab.py)
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python tools/lane_ab.py build/ab_old || exit 1
  timeout -k 10 200 python tools/lane_ab.py build/ab_new || exit 1
done > gpurun_out/lane_ab.txt 2>&1; rc=$?; cat gpurun_out/lane_ab.txt; exit $rc
