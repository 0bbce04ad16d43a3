#!/bin/bash
# the armed-call tests, the armed/plain A/B on C2 (tools/arm_ab.py), then the GPU suite
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-arm1}
timeout -k 10 300 python -u -m pytest tests/test_gpu_arm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_arm_pytest.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_arm_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/arm_ab.py ${AB_TREES:-1000} > gpurun_out/${TAG}_ab.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/${TAG}_ab.txt
[ $rc -eq 0 ] || exit $rc
if [ "${FULL:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  tail -5 gpurun_out/${TAG}_pytest.log
fi
exit $rc
