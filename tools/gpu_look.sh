#!/bin/bash
# the -m lookahead and chained calls on the GPU: chain tests, CLI tests, then the reference's
# example command timed with and without them
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_cli.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/look_pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/look_pytest.log; exit 1; }
tail -3 gpurun_out/look_pytest.log
timeout -k 10 300 python -u tools/example_mp_time.py > gpurun_out/example_mp_time.json 2> gpurun_out/example_mp_time.err || { echo "example_mp_time failed"; tail -20 gpurun_out/example_mp_time.err; exit 1; }
cat gpurun_out/example_mp_time.err gpurun_out/example_mp_time.json
