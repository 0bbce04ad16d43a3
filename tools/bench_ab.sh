#!/bin/bash
# A/B of the headline step between the in-tree engine and a variant copied next to it (GGP_ENGINE_LIB):
#   cp build/ab_NAME/libggp.so gfp_gaussian_process_amd/lib/libggp_NAME.so; AB_LIB=libggp_NAME.so tools/bench_ab.sh
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
Q="--steps 400 --warmup 20 --no-cpu --c4-trees 0 --large-trees 0 --hessian 0 --predict-trees 0 --c5-trees 0 --c3-evals 0 --joints-trees 0 --example-mp 0 --example-parity 0"
: > gpurun_out/benchab.txt
for i in 1 2 3; do
  for L in libggp.so ${AB_LIB:-libggp_tail.so}; do
    GGP_ENGINE_LIB=$L timeout -k 10 120 python bench.py $Q > gpurun_out/benchab_$L.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/benchab_$L.json')); s=d['steps_us']
print('$L', round(d['ms_per_step']*1e3,2), 'events', round(d['roofline']['avg_launch_ms']*1e3,2), 'kernel', round(s['kernel_us']['median'],2), 'mhz', round(s['shader_mhz']['median']))" >> gpurun_out/benchab.txt
  done
done
cat gpurun_out/benchab.txt
