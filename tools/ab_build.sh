#!/bin/bash
# ab_build.sh NAME [INCDIR] -- diagnostic: the engine built into build/ab_NAME/libggp.so, with
# headers from INCDIR (if given) taking precedence over csrc/ (variants for tools/ab_lib.py)
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ab_$1
inc=()
[ -n "$2" ] && inc=(-I"$2")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -shared \
  "${inc[@]}" -Iinclude -Igfp_gaussian_process_amd/csrc -o build/ab_$1/libggp.so gfp_gaussian_process_amd/csrc/ggp_engine.hip -ldl
cp gfp_gaussian_process_amd/lib/libggp_host.so build/ab_$1/
