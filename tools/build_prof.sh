#!/bin/bash
# Instrumented build (per-phase PnP timings via printf) into build/libodo_prof.so:
#   tools/build_prof.sh && python tools/pair_stats.py adaptive-rgbd-localization-mappig_amd/build/libodo_prof.so
set -e
cd "$(dirname "$0")/../adaptive-rgbd-localization-mappig_amd"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -w"
mkdir -p build/prof
for s in k_extract.hip k_match.hip k_ransac.hip odo_capi.cpp; do
  /opt/rocm/bin/hipcc $F -x hip -c csrc/$s -o build/prof/$s.o &
done
/opt/rocm/bin/hipcc $F -DODO_PNP_PROFILE -x hip -c csrc/k_pnp.hip -o build/prof/k_pnp.hip.o
wait
/opt/rocm/bin/hipcc $F -shared -o build/libodo_prof.so build/prof/*.o
