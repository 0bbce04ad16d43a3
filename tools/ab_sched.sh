#!/bin/bash
# scheduler-strategy A/B (diagnostic): the default engine against builds with
# -mllvm -amdgpu-sched-strategy=<s> under tools/ab_sched/<s>/, alternating, C2 / C4-shard / lane sizes.
# Build each variant first (build_ext's engine line plus the -mllvm option, into
# tools/ab_sched/<s>/libggp.so, with a copy of lib/libggp_host.so beside it).
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  for lib in gfp_gaussian_process_amd/lib tools/ab_sched/max-ilp tools/ab_sched/max-memory-clause; do
    for t in 1000 12500 40000; do
      timeout -k 10 120 python tools/ab_lib.py $lib auto $t || exit 1
    done
  done
done > gpurun_out/sched_ab.txt 2>&1
cat gpurun_out/sched_ab.txt
