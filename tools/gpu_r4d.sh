#!/bin/bash
# round 4, batch d: the ExternalStream teardown diagnostic (one mode per process; a crash is a
# result here, not a failure of the batch), then the new chain-stall / device-set / teardown tests
export TMPDIR=/tmp; mkdir -p gpurun_out/r4d
for m in owner_last owner_sync owner_first; do
  timeout -k 10 120 python3 -u tools/extstream_teardown.py $m > gpurun_out/r4d/ext_$m.log 2>&1
  echo "extstream $m: exit $?" | tee -a gpurun_out/r4d/ext_summary.txt
  tail -2 gpurun_out/r4d/ext_$m.log
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_shards.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "stall or chain or descriptor or collective or cap or minimize" > gpurun_out/r4d/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4d/pytest.log | tail -40; exit $rc
