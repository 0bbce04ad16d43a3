#!/bin/bash
# round 5: the >32-segment smoother test; the lane likelihood's pipelined row loads (lib vs ab_l);
# the lane-pair smoother's LDS parameter rows and pipelined row loads (ab_l vs ab_p, 12.5k trees)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "many_segments" -x -v -s --timeout 200 --timeout-method thread > gpurun_out/manyseg.log 2>&1 || { tail -30 gpurun_out/manyseg.log; exit 1; }
tail -3 gpurun_out/manyseg.log
bash tools/lane_prod_ab.sh gfp_gaussian_process_amd/lib tools/ab_l || exit 1
for i in 1 2; do for d in tools/ab_l tools/ab_p; do timeout -k 10 200 python tools/smoother_lane_ab.py $d 12500 || exit 1; done; done > gpurun_out/pair_ab2.txt 2>&1 && grep ms gpurun_out/pair_ab2.txt
