#!/bin/bash
# the example's chains against the reference-Dawson totals (tests/golden/oracle_example_refdawson.json)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "reference_dawson or carried_state_chain" -m gpu -x -v -s --timeout 240 --timeout-method thread > gpurun_out/r4j.log 2>&1
rc=$?; grep -E "worst rel|passed|failed|Error" gpurun_out/r4j.log | tail -12; exit $rc
