#!/bin/bash
# joints: the leg's breakdown (tools/joints_breakdown.py), the joints tests, the bench's joints leg
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 python tools/joints_breakdown.py > gpurun_out/joints_breakdown.json 2> gpurun_out/joints_breakdown.err || { tail gpurun_out/joints_breakdown.err; exit 1; }
cat gpurun_out/joints_breakdown.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_joints.py tests/test_gpu_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4k_pytest.log 2>&1 || { tail -30 gpurun_out/r4k_pytest.log; exit 1; }
tail -1 gpurun_out/r4k_pytest.log
timeout -k 10 300 python bench.py --steps 20 --no-cpu --large-trees 0 --predict-trees 0 --hessian 0 --c3-evals 0 --example-mp 0 > gpurun_out/r4k_bench.json 2> gpurun_out/r4k_bench.err || { tail gpurun_out/r4k_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4k_bench.json')); print(json.dumps(d['joints_c5_subset']))"
