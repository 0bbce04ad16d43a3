#!/bin/bash
# The driver's bench command twice per setting (GGP_BENCH_PIN=1: the timed thread on one CPU, the
# default; 0: unpinned), alternating; the host split of each run
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
for pin in 1 0; do
GGP_BENCH_PIN=$pin timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bh_${pin}_$i.json 2> gpurun_out/bh_${pin}_$i.err || { tail -20 gpurun_out/bh_${pin}_$i.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bh_${pin}_$i.json')); s=d['steps_us']
print('pin=$pin C2 %.4g ms/step %.4f launch(events) %.4f calls %d' % (d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['chained_calls']))
print({k: round(v['median'], 2) for k, v in s.items() if isinstance(v, dict)})"
done
done
