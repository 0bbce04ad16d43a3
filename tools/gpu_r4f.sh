#!/bin/bash
# GPU tests on the working tree's engine (lane bodies: contracted + product exponentials), then an
# alternating A/B of HEAD's engine (build/ab_old), the new one (ab_new), the new one with the
# flagged exponentials in the lane kernels (ab_flag) and the new one without contraction (ab_nocon)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r4f.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r4f.log; grep -E "FAILED|Error" gpurun_out/pytest_r4f.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for b in old new flag nocon; do timeout -k 10 200 python tools/lane_ab.py build/ab_$b || exit 1; done
done > gpurun_out/lane_ab_r4f.txt 2>&1; rc2=$?; grep -v amdgpu.ids gpurun_out/lane_ab_r4f.txt; exit $((rc + rc2))
