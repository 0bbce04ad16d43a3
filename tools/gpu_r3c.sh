#!/bin/bash
# round 3, batch c: the multi-rank rehearsal (bench --gpus 2 with the in-process leg in a child
# process), then the CLI -p writer over the whole C5 forest (5e8 rows) through -chunk
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3c_multirank.log 2>&1 || { echo multirank failed; grep -E "Error|assert|FAILED" gpurun_out/r3c_multirank.log | tail -20; exit 1; }
grep -E "passed|failed" gpurun_out/r3c_multirank.log | tail -2
timeout -k 10 900 python -u tools/writer_c5.py 1000000 "" 62500000 > gpurun_out/r3c_writer_c5_full.json 2> gpurun_out/r3c_writer_c5_full.err || { echo writer failed; tail gpurun_out/r3c_writer_c5_full.err; exit 1; }
cat gpurun_out/r3c_writer_c5_full.err gpurun_out/r3c_writer_c5_full.json
