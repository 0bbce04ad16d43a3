#!/bin/bash
# PMC passes for a few (trees, kernel, cpw) configs; each rocprofv3 run bounded by timeout.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
P2="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_LDS"
for cfg in "1000 lane 1" "1000 lane 64" "1000 group 2" "10000 lane 64"; do
  set -- $cfg
  tag="$1_$2_$3"
  timeout -k 10 120 rocprofv3 --pmc $P1 -d gpurun_out/pmc/p1_$tag -o p --output-format csv -- python3 tools/pmc_probe.py $1 $2 $3 > /dev/null 2>gpurun_out/pmc/err_p1_$tag.log || exit 1
  timeout -k 10 120 rocprofv3 --pmc $P2 -d gpurun_out/pmc/p2_$tag -o p --output-format csv -- python3 tools/pmc_probe.py $1 $2 $3 > /dev/null 2>gpurun_out/pmc/err_p2_$tag.log || exit 1
done
python3 tools/pmc_summary.py gpurun_out/pmc/p* > gpurun_out/pmc/summary.txt
cat gpurun_out/pmc/summary.txt
