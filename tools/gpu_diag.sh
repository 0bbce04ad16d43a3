#!/bin/bash
# Diagnostics of the C2 wave kernel on the GPU box (build/diag/* cross-compiled beforehand from
# tools/stamp_group.hip and tools/timeline.hip): the launch timeline, per-stage stamps at 1000 and
# 512 trees.  Outputs under gpurun_out/diag/.  Usage: tools/gpu_diag.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-diag}
mkdir -p gpurun_out/diag
timeout -k 10 120 build/diag/timeline 1000 200 5 > gpurun_out/diag/${TAG}_timeline_c2.txt 2>&1 || { echo timeline failed; tail -5 gpurun_out/diag/${TAG}_timeline_c2.txt; exit 1; }
timeout -k 10 120 build/diag/stamp_group 1000 3 > gpurun_out/diag/${TAG}_stamps_c2.txt 2>&1 || { echo stamps failed; exit 1; }
timeout -k 10 120 build/diag/stamp_group 512 3 > gpurun_out/diag/${TAG}_stamps_512.txt 2>&1 || { echo stamps 512 failed; exit 1; }
cat gpurun_out/diag/${TAG}_timeline_c2.txt gpurun_out/diag/${TAG}_stamps_c2.txt gpurun_out/diag/${TAG}_stamps_512.txt
