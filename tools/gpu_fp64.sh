#!/bin/bash
# FP64 VALU counters of the C2 bench's kernels (one PMC pass, bounded); the path's real bound
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06}
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc64_${TAG} -o p --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --large-trees 0 --predict-trees 0 > /dev/null 2> gpurun_out/pmc64_${TAG}.err || { echo "pmc fp64 failed"; tail -20 gpurun_out/pmc64_${TAG}.err; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc64_${TAG} > gpurun_out/pmc64_${TAG}.txt
cat gpurun_out/pmc64_${TAG}.txt
