#!/bin/bash
# the chained objective on the GPU: its tests, the CLI tests (Hessian and scan go through it),
# then the timing against call-by-call (tools/chain_time.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_cli.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/chain_pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/chain_pytest.log; exit 1; }
tail -3 gpurun_out/chain_pytest.log
timeout -k 10 300 python -u tools/chain_time.py > gpurun_out/chain_time.json 2> gpurun_out/chain_time.err || { echo "chain_time failed"; tail -20 gpurun_out/chain_time.err; exit 1; }
cat gpurun_out/chain_time.err gpurun_out/chain_time.json
