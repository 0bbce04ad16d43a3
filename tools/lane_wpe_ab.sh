set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python tools/lane_wpe_ab.py gfp_gaussian_process_amd/lib || exit 1
  timeout -k 10 200 python tools/lane_wpe_ab.py tools/ab_wpe || exit 1
done > gpurun_out/wpe_ab.txt 2>&1
cat gpurun_out/wpe_ab.txt
