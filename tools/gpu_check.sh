#!/bin/bash
# One GPU-box session for a round-6 build: the GPU test suite, the driver's bench command, the host
# split probe and the C2 diagnostics (tools/gpu_diag.sh).  A test failure (pytest rc 1) does not stop
# the measurements; a fault, abort or time limit (rc >= 124 or a signal) stops everything after it.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r6}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -6 gpurun_out/${TAG}_pytest.log
[ $rc -le 1 ] || { echo "pytest rc=$rc: stopping"; exit $rc; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json'))
s=d['steps_us']
print('C2 %.4g ms/step %.4f launch(events) %.4f' % (d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms']))
print({k: round(v['median'], 2) for k, v in s.items() if isinstance(v, dict)})
print('large', d.get('large_forest', {}).get('ms_per_eval'), 'predict', d.get('predict', {}).get('ms_per_predict'), 'c4', d.get('c4_strong', {}).get('ms_per_eval'))"
timeout -k 10 120 build/diag/launch_latency > gpurun_out/${TAG}_launch_latency.txt 2>&1 && cat gpurun_out/${TAG}_launch_latency.txt || exit 1
tools/gpu_diag.sh ${TAG} > /dev/null && tail -40 gpurun_out/diag/${TAG}_timeline_c2.txt && head -14 gpurun_out/diag/${TAG}_stamps_c2.txt && head -14 gpurun_out/diag/${TAG}_stamps_512.txt
exit $rc
