#!/bin/bash
# BASELINE configs[4] at full size on one GPU (tools/c5_full.py), under its own limit
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/c5_full.py > gpurun_out/c5_full.json 2> gpurun_out/c5_full.err || { echo c5_full failed; tail -20 gpurun_out/c5_full.err; exit 1; }
cat gpurun_out/c5_full.json
