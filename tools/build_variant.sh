#!/bin/bash
# Build a variant of libodo_hip.so with extra compile flags for A/B runs:
#   tools/build_variant.sh NAME "-DODO_WAVE_PRIO=0"
#     ->  adaptive-rgbd-localization-mappig_amd/build_NAME/libodo_hip.so
# (load it with ODO_LIB=adaptive-rgbd-localization-mappig_amd/build_NAME/libodo_hip.so).
# The source list and flags come from the package Makefile (its variant
# target), linked with --no-undefined. Add -DODO_TUNING to read the
# measurement knobs (ODO_SKIP, ODO_SCHED, ...) from the environment.
set -e
NAME=$1; EXTRA=$2
make -j8 -C "$(dirname "$0")/../adaptive-rgbd-localization-mappig_amd" variant NAME="$NAME" EXTRA="$EXTRA"
