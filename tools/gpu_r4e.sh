#!/bin/bash
# round 4, batch e: the engine-before-torch diagnostic, the C5-shaped -j test, the teardown-order
# collective tests, and a bench run with the new C3 / joints legs
export TMPDIR=/tmp; mkdir -p gpurun_out/r4e
timeout -k 10 120 python3 -u tools/two_runtimes.py > gpurun_out/r4e/two_runtimes.log 2>&1; echo "two_runtimes exit $?"; tail -4 gpurun_out/r4e/two_runtimes.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_joints.py tests/test_gpu_parity.py -x -v -s --timeout 600 --timeout-method thread -k "c5_shape or collective" > gpurun_out/r4e/pytest.log 2>&1 || { grep -E "PASSED|FAILED|Error|assert" gpurun_out/r4e/pytest.log | tail -20; exit 1; }
grep -E "PASSED|FAILED|C5-shaped|collective path" gpurun_out/r4e/pytest.log | tail -10
timeout -k 10 600 python -u bench.py --steps 50 --no-cpu --example-mp 0 --predict-trees 0 --large-trees 0 --hessian 0 > gpurun_out/r4e/bench.json 2> gpurun_out/r4e/bench.err || { tail -20 gpurun_out/r4e/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4e/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d.get('c3_minimize')), json.dumps(d.get('joints_c5_subset')))"
