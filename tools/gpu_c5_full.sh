#!/bin/bash
# the CLI writer tests (multi-span -p byte test), then BASELINE configs[4] at full size on one GPU
# (tools/c5_full.py); each step under its own limit
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cli.py -k "not joints" -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/c5_pytest.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/c5_pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/c5_pytest.log | tail -2
timeout -k 10 900 python -u tools/c5_full.py > gpurun_out/c5_full.json 2> gpurun_out/c5_full.err || { echo c5_full failed; tail -20 gpurun_out/c5_full.err; exit 1; }
cat gpurun_out/c5_full.json
