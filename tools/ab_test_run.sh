#!/bin/bash
# parity tests of the working tree's engine, then tools/ab_run.sh on the given variants
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > gpurun_out/abt_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/abt_pytest.log
[ $rc -le 1 ] || exit $rc
tools/ab_run.sh "$@"
