#!/bin/bash
# the combine fused into the backward pass: the smoother/combine GPU tests, then the C5-shard A/B
# (tools/lane_ab_c5.py) of the fused build (ab_fused) against the separate combine (ab_new = r33)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "predict or combine or smoother" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4l_pytest.log 2>&1 || { tail -30 gpurun_out/r4l_pytest.log; exit 1; }
tail -1 gpurun_out/r4l_pytest.log
for i in 1 2; do
  for b in new fused; do timeout -k 10 200 python tools/lane_ab_c5.py build/ab_$b || exit 1; done
done > gpurun_out/r4l.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r4l.txt; exit $rc
