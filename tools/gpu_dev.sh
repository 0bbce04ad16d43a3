#!/bin/bash
# development round on the GPU box: the GPU suite, a C2 bench, the example -m -p leg, wave-kernel
# stage stamps.  Every GPU step under its own time limit; stops at the first failure.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dev_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/dev_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --no-cpu --large-trees 0 --predict-trees 0 --hessian 0 > gpurun_out/dev_bench.json 2> gpurun_out/dev_bench.err || { echo bench failed; tail gpurun_out/dev_bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/dev_bench.json')); print('value %.4g ms/step %.4f kernel %.4f' % (d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])); print(json.dumps(d.get('example_mp')))"
timeout -k 10 120 tools/stamp_group 1000 3 > gpurun_out/stamps.txt 2>&1; cat gpurun_out/stamps.txt
