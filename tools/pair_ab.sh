set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2 3; do for d in build/ab_old gfp_gaussian_process_amd/lib; do timeout -k 10 120 python tools/pair_ab.py $d || exit 1; done; done > gpurun_out/pair_ab.txt 2>&1
grep trees gpurun_out/pair_ab.txt
