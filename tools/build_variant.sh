#!/bin/bash
# Build a variant of libodo_hip.so with extra compile flags for A/B runs:
#   tools/build_variant.sh NAME "-DODO_WAVE_PRIO=0"  ->  build/libodo_NAME.so
# (load it with ODO_LIB=adaptive-rgbd-localization-mappig_amd/build/libodo_NAME.so)
set -e
NAME=$1; EXTRA=$2
cd "$(dirname "$0")/../adaptive-rgbd-localization-mappig_amd"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -w $EXTRA"
mkdir -p build/$NAME
for s in k_extract.hip k_finalize.hip k_adaptive.hip k_adaptive_orb.hip k_match.hip k_project.hip k_ransac.hip k_pnp.hip odo_capi.cpp; do
  X=""; [ $s = k_match.hip ] && X="-mllvm -amdgpu-mfma-vgpr-form"  # as the Makefile
  /opt/rocm/bin/hipcc $F $X -x hip -c csrc/$s -o build/$NAME/$s.o &
done
wait
/opt/rocm/bin/hipcc $F -shared -o build/libodo_$NAME.so build/$NAME/*.o
