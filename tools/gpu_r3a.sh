#!/bin/bash
# round 3, batch a: the writer/joints GPU tests, then the full-size runs (example -js, the -p
# writer on a C5 shard, the whole C5 forest on one GPU).  Each step under its own limit; stop at
# the first failure.
export TMPDIR=/tmp; mkdir -p gpurun_out
df -h /tmp . > gpurun_out/df.txt 2>&1; cat gpurun_out/df.txt
timeout -k 10 420 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_joints.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r3a_pytest.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/r3a_pytest.log; exit 1; }
grep -E "passed|failed|example full" gpurun_out/r3a_pytest.log | tail -5
timeout -k 10 240 python -u tools/joints_example_full.py > gpurun_out/r3a_joints_full.json 2> gpurun_out/r3a_joints_full.err || { echo joints_full failed; tail gpurun_out/r3a_joints_full.err; exit 1; }
cat gpurun_out/r3a_joints_full.json
timeout -k 10 420 python -u tools/writer_c5.py > gpurun_out/r3a_writer.json 2> gpurun_out/r3a_writer.err || { echo writer failed; tail gpurun_out/r3a_writer.err; exit 1; }
cat gpurun_out/r3a_writer.json
