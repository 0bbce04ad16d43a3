#!/bin/bash
# Cross-compile the diagnostic binaries tools/gpu_diag.sh and tools/gpu_check.sh run (build/diag/,
# git-ignored, travels to the GPU box): the timeline and stamps builds of the engine, the launch
# latency probe.  Run after any change to ggp_engine.hip.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/diag
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off"
L="-Lgfp_gaussian_process_amd/lib -lggp_host -Wl,-rpath,\$ORIGIN/../../gfp_gaussian_process_amd/lib"
/opt/rocm/bin/hipcc $F -Iinclude -Igfp_gaussian_process_amd/csrc -o build/diag/timeline tools/timeline.hip $L &
/opt/rocm/bin/hipcc $F -Iinclude -Igfp_gaussian_process_amd/csrc -o build/diag/stamp_group tools/stamp_group.hip $L &
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -o build/diag/launch_latency tools/launch_latency.hip \
    -Lgfp_gaussian_process_amd/lib -lggp -lggp_host -Wl,-rpath,\$ORIGIN/../../gfp_gaussian_process_amd/lib &
wait
ls -la build/diag
