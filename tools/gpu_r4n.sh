#!/bin/bash
# the lane kernels' row loads issued before the propagation (ab_new) against HEAD (ab_old): C5 shard
# (tools/lane_ab_c5.py), C4 shard + 20k-tree smoother (tools/lane_ab.py); then the parity tests
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  for b in old new; do
    timeout -k 10 200 python tools/lane_ab_c5.py build/ab_$b || exit 1
    timeout -k 10 200 python tools/lane_ab.py build/ab_$b || exit 1
  done
done > gpurun_out/r4n.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r4n.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_joints.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4n_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r4n_pytest.log; exit $rc
