#!/bin/bash
# Build an A/B variant of the engine (diagnostic): tools/ab_build.sh NAME [REV]
#   build/ab_NAME/libggp.so and build/diag/stamp_NAME from ggp_engine.hip as in the working tree,
#   or as in git revision REV (the other sources from the working tree)
set -e
cd "$(dirname "$0")/.."
NAME=$1; REV=$2
SRC=gfp_gaussian_process_amd/csrc
TMP=$(mktemp -d)
if [ -n "$REV" ]; then git show "$REV:$SRC/ggp_engine.hip" > $TMP/ggp_engine.hip; else cp $SRC/ggp_engine.hip $TMP/; fi
mkdir -p build/ab_$NAME build/diag
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -cuid=ggp_engine"
/opt/rocm/bin/hipcc $F -fPIC -shared -Iinclude -I$SRC -o build/ab_$NAME/libggp.so $TMP/ggp_engine.hip -ldl &
/opt/rocm/bin/hipcc $F -I$TMP -Iinclude -I$SRC -o build/diag/stamp_$NAME tools/stamp_group.hip \
    -Lgfp_gaussian_process_amd/lib -lggp_host -Wl,-rpath,'$ORIGIN/../../gfp_gaussian_process_amd/lib' &
wait
cp gfp_gaussian_process_amd/lib/libggp_host.so build/ab_$NAME/ 2>/dev/null || true
rm -rf $TMP
echo built build/ab_$NAME build/diag/stamp_$NAME
