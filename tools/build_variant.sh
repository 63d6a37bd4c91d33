#!/usr/bin/env bash
# Experiment variant of libmarlsched.so (extra compiler defines) into tools/_variants/<name>/;
# load it with MARLSCHED_LIB=tools/_variants/<name>/libmarlsched.so (measurement runs only).
# Usage: bash tools/build_variant.sh <name> "<extra hipcc flags>"
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
NAME="$1"
OUTDIR="${HERE}/_variants/${NAME}"
mkdir -p "${OUTDIR}"
MS_OUT="${OUTDIR}/libmarlsched.so" MS_OBJDIR="${OUTDIR}/obj" MS_EXTRA_FLAGS="$2" bash "${HERE}/../marl-scheduling_amd/build.sh"
