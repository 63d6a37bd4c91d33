#!/usr/bin/env bash
# Builds libmarlsched.so (gfx950) in-tree: the HIP kernels + the C ABI.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUT="${HERE}/libmarlsched.so"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
ARCH="${MS_OFFLOAD_ARCH:-gfx950}"
FLAGS=(-O3 -std=c++17 -fPIC --offload-arch="${ARCH}" -Wall -Wno-unused-function
       -I"${HERE}/../include")
OBJDIR="${HERE}/build"
mkdir -p "${OBJDIR}"
objs=()
for src in env_kernels.hip policy_kernels.hip ppo_kernels.hip agg_kernels.hip capi.cpp; do
  obj="${OBJDIR}/${src%.*}.o"
  if [[ ! -f "${obj}" || "${HERE}/csrc/${src}" -nt "${obj}" || "${HERE}/csrc/ms_layout.h" -nt "${obj}" || "${HERE}/csrc/ms_ppo.h" -nt "${obj}" || "${HERE}/../include/marlsched.h" -nt "${obj}" ]]; then
    # the env round reproduces Python's float64 arithmetic: no contraction there; the policy
    # and PPO kernels follow torch's f32 (which fuses freely) within tolerance: fma allowed
    contract=(-ffp-contract=off)
    [[ "${src}" == policy_kernels.hip || "${src}" == ppo_kernels.hip ]] && contract=(-ffp-contract=fast)
    if [[ "${src}" == *.cpp ]]; then
      "${HIPCC}" "${FLAGS[@]}" "${contract[@]}" -x hip -c "${HERE}/csrc/${src}" -o "${obj}"
    else
      "${HIPCC}" "${FLAGS[@]}" "${contract[@]}" -c "${HERE}/csrc/${src}" -o "${obj}"
    fi
  fi
  objs+=("${obj}")
done
"${HIPCC}" -shared -fPIC --offload-arch="${ARCH}" -o "${OUT}" "${objs[@]}"
echo "${OUT}"
