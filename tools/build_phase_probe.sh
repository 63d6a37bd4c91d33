#!/usr/bin/env bash
# Profiling-only build: libmarlsched with per-phase cycle counters in k_env_step (MS_PHASE_TIMING, see
# env_kernels.hip), all sources as build.sh compiles them. Output: tools/_probe[_lpeN]/libmarlsched_probe.so.
# The product library (marl-scheduling_amd/libmarlsched.so) is never built this way.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUT="${HERE}/_probe${1:+_lpe$1}"
mkdir -p "${OUT}"
MS_EXTRA_FLAGS="-DMS_PHASE_TIMING ${1:+-DMS_MIN_LPE=$1}" MS_OUT="${OUT}/libmarlsched_probe.so" MS_OBJDIR="${OUT}/obj" \
  bash "${HERE}/../marl-scheduling_amd/build.sh"
