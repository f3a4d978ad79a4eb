#!/bin/bash
# Instrumented build (per-phase PnP timings via printf) into build_prof/libodo_hip.so:
#   tools/build_prof.sh && python tools/pair_stats.py adaptive-rgbd-localization-mappig_amd/build_prof/libodo_hip.so
exec "$(dirname "$0")/build_variant.sh" prof "-DODO_TUNING -DODO_PNP_PROFILE"
