#!/bin/bash
# ab_pair.sh A B [ROUNDS=3] -- diagnostic: alternating tools/ab_lib.py timings of build/ab_A and
# build/ab_B on C2 (auto schedule)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in $(seq 1 ${3:-3}); do
  timeout -k 10 120 python tools/ab_lib.py build/ab_$1 auto 1000 || exit 1
  timeout -k 10 120 python tools/ab_lib.py build/ab_$2 auto 1000 || exit 1
done 2>&1 | tee gpurun_out/ab_pair.txt
