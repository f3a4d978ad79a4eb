#!/bin/bash
# Instrumented build (per-phase PnP timings via printf) into build/libodo_prof.so:
#   tools/build_prof.sh && python tools/pair_stats.py adaptive-rgbd-localization-mappig_amd/build/libodo_prof.so
exec "$(dirname "$0")/build_variant.sh" prof "-DODO_PNP_PROFILE"
