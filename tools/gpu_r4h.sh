#!/bin/bash
# parity margins (tools/parity_margin.py) of the engine before (build/ab_old = 532ab38) and after
# (build/ab_new) the lane-body change
export TMPDIR=/tmp; mkdir -p gpurun_out
{ timeout -k 10 300 python tools/parity_margin.py build/ab_old && timeout -k 10 300 python tools/parity_margin.py build/ab_new; } > gpurun_out/r4h.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r4h.txt; exit $rc
