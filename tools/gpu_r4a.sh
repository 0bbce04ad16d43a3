#!/bin/bash
# round 4, batch a: per-stage s_memtime stamps of k_loglik_wave on the shipped sources (GGP_STAMPS
# build, tools/stamp_group) for C2 and the C5 tree shape, then the PMC instruction mix of one pass.
export TMPDIR=/tmp; mkdir -p gpurun_out/stamps
timeout -k 10 120 tools/stamp_group 1000 3 200 > gpurun_out/stamps/r4_c2.txt 2>&1 || { echo stamp c2 failed; cat gpurun_out/stamps/r4_c2.txt; exit 1; }
timeout -k 10 120 tools/stamp_group 1000 3 500 > gpurun_out/stamps/r4_c5shape.txt 2>&1 || { echo stamp c5 failed; exit 1; }
cat gpurun_out/stamps/r4_c2.txt gpurun_out/stamps/r4_c5shape.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 -d gpurun_out/stamps/pmc -o p --output-format csv -- python3 tools/pmc_probe.py 1000 wave 1 > gpurun_out/stamps/pmc.out 2> gpurun_out/stamps/pmc.err || { tail -5 gpurun_out/stamps/pmc.err; exit 1; }
python3 tools/pmc_summary.py gpurun_out/stamps/pmc
