#!/bin/bash
# Where the lane schedule's cycles go (PMC, separate passes): the likelihood's k_loglik_level on a
# 40k-tree forest (40k-cell roots, 80k-cell daughters: lane schedule) and the -p lane smoother
# (k_fwd_level / k_bwd_level) on 40k C5-shaped trees.  python3 tools/pmc_summary.py prints per kernel.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/lstall
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
P2="SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VALU"
for p in 1 2; do
  eval "C=\$P$p"
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/lstall/l$p -o p --output-format csv -- python3 tools/pmc_probe.py 40000 lane 64 3 > gpurun_out/lstall/l$p.out 2> gpurun_out/lstall/l$p.err || { tail -5 gpurun_out/lstall/l$p.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/lstall/s$p -o p --output-format csv -- python3 tools/combine_workload.py 40000 > gpurun_out/lstall/s$p.out 2> gpurun_out/lstall/s$p.err || { tail -5 gpurun_out/lstall/s$p.err; exit 1; }
done
for p in 1 2; do python3 tools/pmc_summary.py gpurun_out/lstall/l$p; python3 tools/pmc_summary.py gpurun_out/lstall/s$p; done > gpurun_out/lstall/summary.txt
grep -A9 "k_loglik_level\|k_fwd_level\|k_bwd_level" gpurun_out/lstall/summary.txt | head -80
