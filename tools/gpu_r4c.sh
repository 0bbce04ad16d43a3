#!/bin/bash
# round 4, batch c: timeline of the new build, alternating A/B against build/ab_old (HEAD), then
# the wave / chain / shard parity tests
export TMPDIR=/tmp; mkdir -p gpurun_out
gunzip -c tests/golden/example_input.csv.gz > /tmp/ex.csv; (timeout -k 10 60 tools/timeline 1000 200 1 && timeout -k 10 60 tools/timeline 0 /tmp/ex.csv 1 tests/golden/example_csv_config.txt) > gpurun_out/r4c_timeline.txt 2>&1 || { echo timeline failed; cat gpurun_out/r4c_timeline.txt; exit 1; }
grep -E "counts|eval" gpurun_out/r4c_timeline.txt
for i in 1 2 3; do
  timeout -k 10 120 python tools/ab_lib.py build/ab_old auto 1000 || exit 1
  timeout -k 10 120 python tools/ab_lib.py gfp_gaussian_process_amd/lib auto 1000 || exit 1
done > gpurun_out/r4c_ab.txt 2>&1 || { cat gpurun_out/r4c_ab.txt; exit 1; }
for i in 1 2; do
  timeout -k 10 120 python tools/ab_lib.py build/ab_old auto 0 || exit 1
  timeout -k 10 120 python tools/ab_lib.py gfp_gaussian_process_amd/lib auto 0 || exit 1
done >> gpurun_out/r4c_ab.txt 2>&1 || { cat gpurun_out/r4c_ab.txt; exit 1; }
cat gpurun_out/r4c_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_shards.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r4c_pytest.log; exit $rc
