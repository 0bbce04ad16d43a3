set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/multirank.log 2>&1 || { tail -40 gpurun_out/multirank.log; exit 1; }
grep -h "collective:\|passed\|failed" gpurun_out/multirank.log
