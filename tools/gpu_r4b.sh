#!/bin/bash
# round 4, batch b: where a C2 wave-step's cycles go (PMC, separate passes), at 1000 trees (two
# active waves per SIMD in the last quarter of the rows) and 512 trees (one wave per SIMD)
export TMPDIR=/tmp; mkdir -p gpurun_out/r4b
for T in 1000 512; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/r4b/p1_$T -o p --output-format csv -- python3 tools/pmc_probe.py $T wave 1 > gpurun_out/r4b/p1_$T.out 2> gpurun_out/r4b/p1_$T.err || { tail -5 gpurun_out/r4b/p1_$T.err; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU -d gpurun_out/r4b/p2_$T -o p --output-format csv -- python3 tools/pmc_probe.py $T wave 1 > gpurun_out/r4b/p2_$T.out 2> gpurun_out/r4b/p2_$T.err || { tail -5 gpurun_out/r4b/p2_$T.err; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r4b/p1_$T > gpurun_out/r4b/sum_$T.txt
python3 tools/pmc_summary.py gpurun_out/r4b/p2_$T >> gpurun_out/r4b/sum_$T.txt
done
grep -A9 "k_loglik_wave" gpurun_out/r4b/sum_1000.txt gpurun_out/r4b/sum_512.txt
