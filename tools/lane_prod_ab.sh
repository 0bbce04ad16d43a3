set -o pipefail
# lane-schedule variants against the shipped engine, alternating (tools/lane_wpe_ab.py prints the
# times, the total and a hash of 400k combined -p rows): python tools/lane_wpe_ab.py LIB_DIR
# usage: bash tools/lane_prod_ab.sh DIR...   (default: the shipped lib, tools/ab_p1, tools/ab_p2)
export TMPDIR=/tmp; mkdir -p gpurun_out
DIRS=${*:-"gfp_gaussian_process_amd/lib tools/ab_p1 tools/ab_p2"}
for i in 1 2; do
  for d in $DIRS; do
    timeout -k 10 200 python tools/lane_wpe_ab.py $d || exit 1
  done
done > gpurun_out/prod_ab.txt 2>&1
grep ms gpurun_out/prod_ab.txt
