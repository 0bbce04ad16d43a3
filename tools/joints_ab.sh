set -o pipefail
# usage: bash tools/joints_ab.sh DIR...  (alternating; each DIR holds libggp.so + libggp_host.so)
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2 3; do for d in "$@"; do timeout -k 10 120 python tools/joints_ab.py $d || exit 1; done; done > gpurun_out/joints_ab.txt 2>&1
grep joints gpurun_out/joints_ab.txt
