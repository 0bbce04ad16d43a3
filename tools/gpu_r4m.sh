#!/bin/bash
# HBM traffic of the -p leg's kernels on a C5 shard (bench.py predict leg only): FETCH_SIZE and
# WRITE_SIZE passes, the fused combine (default) and the separate one (GGP_COMBINE_FUSED=0)
export TMPDIR=/tmp; mkdir -p gpurun_out
ARGS="--steps 1 --warmup 1 --no-cpu --large-trees 0 --hessian 0 --c3-evals 0 --joints-trees 0 --example-mp 0"
for mode in fused sep; do
  if [ $mode = sep ]; then export GGP_COMBINE_FUSED=0; fi
  timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcpf_$mode -o p --output-format csv -- python3 bench.py $ARGS > /dev/null 2> gpurun_out/pmcpf_$mode.err || { echo "fetch $mode failed"; tail -5 gpurun_out/pmcpf_$mode.err; exit 1; }
  timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcpw_$mode -o p --output-format csv -- python3 bench.py $ARGS > /dev/null 2> gpurun_out/pmcpw_$mode.err || { echo "write $mode failed"; tail -5 gpurun_out/pmcpw_$mode.err; exit 1; }
  python3 tools/pmc_traffic.py gpurun_out/pmcpf_$mode gpurun_out/pmcpw_$mode gpurun_out/predict_traffic_$mode.json > /dev/null
done
cat gpurun_out/predict_traffic_fused.json gpurun_out/predict_traffic_sep.json
