#!/bin/bash
# round 3, batch b: the CLI writer tests (byte-exact text), then the writer and -js timings again
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3b_pytest.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/r3b_pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/r3b_pytest.log | tail -2
timeout -k 10 420 python -u tools/writer_c5.py > gpurun_out/r3b_writer.json 2> gpurun_out/r3b_writer.err || { echo writer failed; tail gpurun_out/r3b_writer.err; exit 1; }
cat gpurun_out/r3b_writer.json
timeout -k 10 240 python -u tools/joints_example_full.py > gpurun_out/r3b_joints_full.json 2> gpurun_out/r3b_joints_full.err || { echo joints_full failed; tail gpurun_out/r3b_joints_full.err; exit 1; }
cat gpurun_out/r3b_joints_full.json
