#!/usr/bin/env bash
# Profiling-only build: libmarlsched with per-phase cycle counters in k_env_step
# (MS_PHASE_TIMING, see env_kernels.hip). Output: tools/_probe/libmarlsched_probe.so.
# The product library (marl-scheduling_amd/libmarlsched.so) is never built this way.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
SRC="${HERE}/../marl-scheduling_amd/csrc"
OUT="${HERE}/_probe${1:+_lpe$1}"
LPE_DEF=(${1:+-DMS_MIN_LPE=$1})
mkdir -p "${OUT}"
FLAGS=(-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I"${HERE}/../include")
/opt/rocm/bin/hipcc "${FLAGS[@]}" -DMS_PHASE_TIMING "${LPE_DEF[@]}" -c "${SRC}/env_kernels.hip" -o "${OUT}/env_kernels.o"
/opt/rocm/bin/hipcc "${FLAGS[@]}" -ffp-contract=fast -mllvm -amdgpu-sched-strategy=max-ilp -c "${SRC}/policy_kernels.hip" -o "${OUT}/policy_kernels.o"
/opt/rocm/bin/hipcc "${FLAGS[@]}" -ffp-contract=fast -c "${SRC}/returns_kernels.hip" -o "${OUT}/returns_kernels.o"
/opt/rocm/bin/hipcc "${FLAGS[@]}" -ffp-contract=on -c "${SRC}/ppo_kernels.hip" -o "${OUT}/ppo_kernels.o"
/opt/rocm/bin/hipcc "${FLAGS[@]}" -c "${SRC}/agg_kernels.hip" -o "${OUT}/agg_kernels.o"
/opt/rocm/bin/hipcc "${FLAGS[@]}" -c "${SRC}/dqn_kernels.hip" -o "${OUT}/dqn_kernels.o"
/opt/rocm/bin/hipcc "${FLAGS[@]}" -x hip -c "${SRC}/capi.cpp" -o "${OUT}/capi.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "${OUT}/libmarlsched_probe.so" "${OUT}"/*.o
echo "${OUT}/libmarlsched_probe.so"
