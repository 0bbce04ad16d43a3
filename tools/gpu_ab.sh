#!/bin/bash
# A/B of the wave kernels on C2 (parity subset first); diagnostic
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "not c4_shard" --timeout 120 --timeout-method thread > gpurun_out/w2_parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/w2_parity.log; [ $rc -eq 0 ] || exit 1
for v in 0 1 0 1; do
GGP_WAVE_V1=$v timeout -k 10 200 python bench.py --no-cpu --large-trees 0 --predict-trees 0 --hessian 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo bench failed; tail gpurun_out/ab_$v.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/ab_$v.json')); print('v1=$v', 'value %.4g ms/step %.4f kernel %.4f' % (d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms']))"
done
timeout -k 10 120 tools/stamp_group 1000 3 > gpurun_out/stamps_w2.txt 2>&1; cat gpurun_out/stamps_w2.txt
