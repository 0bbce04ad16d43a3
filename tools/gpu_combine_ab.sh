#!/bin/bash
# combine A/B (tools/lane_ab.py) then the smoother parity tests on the new build
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python tools/lane_ab.py build/ab_old || exit 1
  timeout -k 10 200 python tools/lane_ab.py build/ab_new || exit 1
done > gpurun_out/combine_ab.txt 2>&1 || { cat gpurun_out/combine_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/combine_ab.txt
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_cli.py tests/test_gpu_joints.py -x -v -s --timeout 400 --timeout-method thread -k "predict or combine or own_noise or joints" > gpurun_out/combine_pytest.log 2>&1; rc=$?
grep -E "^example|^c5_shape|PASSED|FAILED|passed|failed" gpurun_out/combine_pytest.log | tail -40; exit $rc
