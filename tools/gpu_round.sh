#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace + PMC traffic passes.
# Every GPU step is bounded by its own timeout and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o bench --output-format csv -- python3 bench.py --steps 20 --no-cpu --c5-trees 0 --example-parity 0 > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err || { echo "rocprof failed"; tail -20 gpurun_out/prof_${TAG}.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_${TAG} -o p --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --large-trees 0 --predict-trees 0 --hessian 0 --c3-evals 0 --joints-trees 0 --example-mp 0 --c4-trees 0 --c5-trees 0 --example-parity 0 > /dev/null 2> gpurun_out/pmcf_${TAG}.err || { echo "pmc fetch failed"; tail -20 gpurun_out/pmcf_${TAG}.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_${TAG} -o p --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --large-trees 0 --predict-trees 0 --hessian 0 --c3-evals 0 --joints-trees 0 --example-mp 0 --c4-trees 0 --c5-trees 0 --example-parity 0 > /dev/null 2> gpurun_out/pmcw_${TAG}.err || { echo "pmc write failed"; tail -20 gpurun_out/pmcw_${TAG}.err; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmcf_${TAG} gpurun_out/pmcw_${TAG} gpurun_out/traffic_${TAG}.json
mkdir -p profiles && cp gpurun_out/traffic_${TAG}.json profiles/traffic.json
# FP64 work per update (issued: the wave kernel; useful: the lane kernel on full waves), one pass
mkdir -p gpurun_out/pmc64_${TAG}
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmc64_${TAG} -o p --output-format csv -- python3 tools/fp64_workload.py > gpurun_out/pmc64_${TAG}/workload.json 2> gpurun_out/pmc64_${TAG}.err || { echo "pmc fp64 failed"; tail -20 gpurun_out/pmc64_${TAG}.err; exit 1; }
python3 tools/fp64_summary.py gpurun_out/pmc64_${TAG} gpurun_out/fp64_${TAG}.json && cp gpurun_out/fp64_${TAG}.json profiles/fp64_counts.json
timeout -k 10 500 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; cat gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
find gpurun_out/prof_${TAG} -name "*stats*"
