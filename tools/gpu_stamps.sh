#!/bin/bash
# per-stage s_memtime stamps (tools/stamp_group, GGP_STAMPS build) of the wave kernels on C2, and the
# PMC instruction mix of the shipped k_loglik_wave2 (one rocprofv3 pass).  Diagnostic only.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/stamps
timeout -k 10 120 tools/stamp_group 1000 3 > gpurun_out/stamps/w2_c2.txt 2>&1 || { echo stamp w2 failed; cat gpurun_out/stamps/w2_c2.txt; exit 1; }
GGP_WAVE_V1=1 timeout -k 10 120 tools/stamp_group 1000 3 > gpurun_out/stamps/w1_c2.txt 2>&1 || { echo stamp w1 failed; exit 1; }
cat gpurun_out/stamps/w2_c2.txt gpurun_out/stamps/w1_c2.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 -d gpurun_out/stamps/pmc -o p --output-format csv -- python3 tools/pmc_probe.py 1000 wave 1 > gpurun_out/stamps/pmc.out 2> gpurun_out/stamps/pmc.err || { tail -5 gpurun_out/stamps/pmc.err; exit 1; }
python3 tools/pmc_summary.py gpurun_out/stamps/pmc
