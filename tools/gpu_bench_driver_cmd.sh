#!/bin/bash
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bh_$i.json 2> gpurun_out/bh_$i.err || { tail -20 gpurun_out/bh_$i.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bh_$i.json')); s=d['steps_us']
print('C2 %.4g ms/step %.4f launch(events) %.4f calls %d' % (d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['chained_calls']))
print({k: round(v['median'], 2) for k, v in s.items() if isinstance(v, dict)})"
done
