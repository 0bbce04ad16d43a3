#!/bin/bash
# quick GPU check after a kernel change: parity subset + C2 bench (no CPU leg)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/quick_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/quick_pytest.log; exit 1; }
tail -2 gpurun_out/quick_pytest.log
timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err || { echo "bench failed"; tail -20 gpurun_out/quick_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/quick_bench.json'))
print('C2 value %.4g ms/step %.4f' % (d['value'], d['ms_per_step']), d['roofline']['per_kernel_ms'], 'large', d.get('large_forest', {}).get('updates_per_s_per_gpu'))"
