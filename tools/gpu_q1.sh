#!/bin/bash
# the GPU suite (lane queue first), then the queue A/B on C4 (tools/queue_ab.py)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-q1}
timeout -k 10 900 python -u -m pytest tests/test_gpu_lane_queue.py tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/queue_ab.py > gpurun_out/${TAG}_ab.txt 2>&1; rc2=$?
grep -v amdgpu.ids gpurun_out/${TAG}_ab.txt
exit $((rc | rc2))
