set -o pipefail
# lane-smoother builds alternating: bash tools/smoother_lane_ab.sh DIR...
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2 3; do
  for d in "$@"; do
    timeout -k 10 200 python tools/smoother_lane_ab.py $d || exit 1
  done
done > gpurun_out/smoother_ab.txt 2>&1
grep ms gpurun_out/smoother_ab.txt
