#!/bin/bash
# The FP64 PMC pass alone (tools/gpu_round.sh's), for a re-stamp of profiles/fp64_counts.json
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-fp64}
mkdir -p gpurun_out/pmc64_${TAG}
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmc64_${TAG} -o p --output-format csv -- python3 tools/fp64_workload.py > gpurun_out/pmc64_${TAG}/workload.json 2> gpurun_out/pmc64_${TAG}.err || { echo "pmc fp64 failed"; tail -20 gpurun_out/pmc64_${TAG}.err; exit 1; }
python3 tools/fp64_summary.py gpurun_out/pmc64_${TAG} gpurun_out/fp64_${TAG}.json && python3 -c "
import json; d=json.load(open('gpurun_out/fp64_${TAG}.json')); print(d['useful_flops_per_update'], d['issued_flops_per_update'])"
