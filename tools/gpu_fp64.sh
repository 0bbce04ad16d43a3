#!/bin/bash
# the FP64 counter pass alone (tools/fp64_workload.py: C2 wave, lane, the large_forest and predict
# legs), then one bench run that reads it
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-fp}
mkdir -p gpurun_out/pmc64_${TAG}
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmc64_${TAG} -o p --output-format csv -- python3 tools/fp64_workload.py > gpurun_out/pmc64_${TAG}/workload.json 2> gpurun_out/pmc64_${TAG}.err || { echo "pmc fp64 failed"; tail -20 gpurun_out/pmc64_${TAG}.err; exit 1; }
python3 tools/fp64_summary.py gpurun_out/pmc64_${TAG} gpurun_out/fp64_${TAG}.json > /dev/null && cp gpurun_out/fp64_${TAG}.json profiles/fp64_counts.json
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/fp64_${TAG}.json
cat gpurun_out/bench_${TAG}.json
