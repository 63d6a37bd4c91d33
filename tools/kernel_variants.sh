#!/usr/bin/env bash
# rocprofv3 kernel-time stats of one cfg3 PPO iteration (bench.py --steps 1, training rollout only) under
# library variants (tools/_variants/<name>/libmarlsched.so) and the in-tree library, one box (via gpurun).
# Usage: bash tools/kernel_variants.sh <tag> "<variant names>" [kernel name regex for the summary]
set -euo pipefail
export MARLSCHED_LENIENT_ABI=1  # variants built at an older ABI load without the newer entry points
TAG="$1"; VARS="$2"; RX="${3:-k_ppo_grad|k_act|k_env_step|k_key|k_unit}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for v in new $VARS; do
  if [[ "$v" == new ]]; then unset MARLSCHED_LIB; else export MARLSCHED_LIB="$R/tools/_variants/$v/libmarlsched.so"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/$v" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-step-kernel > "$O/$v.json" 2> "$O/$v.err"
  echo "== $v"
  python3 "$R/profiles/summarize.py" "$O/$v"/*/run_kernel_stats.csv 2>/dev/null | grep -E "$RX" || \
    python3 "$R/profiles/summarize.py" "$O/$v/run_kernel_stats.csv" | grep -E "$RX"
done
