#!/bin/bash
# ab_old.sh [REV=HEAD] -- diagnostic: the engine as of REV (ggp_engine.hip and every csrc header
# from git) into build/ab_old/libggp.so, for tools/ab_quick.sh's alternating A/B
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}
src=build/ab_old_src
rm -rf "$src" && mkdir -p "$src" build/ab_old
for f in $(git ls-tree --name-only "$rev" gfp_gaussian_process_amd/csrc/ | grep -E '\.(hip|h|inc)$'); do
  git show "$rev:$f" > "$src/$(basename "$f")"
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -cuid=ggp_engine -shared \
  -Iinclude -I"$src" -o build/ab_old/libggp.so "$src/ggp_engine.hip" -ldl
cp gfp_gaussian_process_amd/lib/libggp_host.so build/ab_old/
