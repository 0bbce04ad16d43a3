set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_joints.py tests/test_gpu_cli.py tests/test_gpu_shards.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/joints_tests.log 2>&1 || { tail -30 gpurun_out/joints_tests.log; exit 1; }
tail -2 gpurun_out/joints_tests.log
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --large-trees 0 --predict-trees 0 --hessian 0 --c3-evals 0 --example-mp 0 --c4-trees 0 --c5-trees 0 --example-parity 0 > gpurun_out/jb.json 2> gpurun_out/jb.err || { tail -5 gpurun_out/jb.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/jb.json').read().splitlines()[-1]); print(d['joints_c5_subset'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/jt -o jt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --large-trees 0 --predict-trees 0 --hessian 0 --c3-evals 0 --example-mp 0 --c4-trees 0 --c5-trees 0 --example-parity 0 > gpurun_out/jt.json 2> gpurun_out/jt.err || { tail -5 gpurun_out/jt.err; exit 1; }
grep -h "joint" gpurun_out/jt/jt_kernel_stats.csv | cut -c1-60,200-400
