set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for n in 2 4 8; do timeout -k 10 120 python tools/node_exchange_bench.py $n 2>/dev/null || exit 1; done > gpurun_out/node_exchange.txt
cat gpurun_out/node_exchange.txt
