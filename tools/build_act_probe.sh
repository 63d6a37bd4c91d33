#!/usr/bin/env bash
# Profiling-only build: libmarlsched with per-phase cycle counters in the paired act kernel (MS_ACT_PROBE, see
# policy_kernels.hip), all sources as build.sh compiles them. Output: tools/_probe_act/libmarlsched.so.
# The product library (marl-scheduling_amd/libmarlsched.so) is never built this way.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUT="${HERE}/_probe_act${1:+_$1}"
mkdir -p "${OUT}"
MS_EXTRA_FLAGS="-DMS_ACT_PROBE ${2:-}" MS_OUT="${OUT}/libmarlsched.so" MS_OBJDIR="${OUT}/obj" \
  bash "${HERE}/../marl-scheduling_amd/build.sh"
