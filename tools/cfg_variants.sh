#!/usr/bin/env bash
# rocprofv3 kernel-time stats of one PPO iteration of a BASELINE config under library variants
# (tools/_variants/<name>/libmarlsched.so) and the in-tree library, one box (via gpurun).
# Usage: bash tools/cfg_variants.sh <tag> <config> "<variant names>" [kernel name regex]
set -euo pipefail
export MARLSCHED_LENIENT_ABI=1  # variants built at an older ABI load without the newer entry points
TAG="$1"; CFG="$2"; VARS="$3"; RX="${4:-k_ppo_grad|k_act|k_env_step}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for v in new $VARS; do
  if [[ "$v" == new ]]; then unset MARLSCHED_LIB; else export MARLSCHED_LIB="$R/tools/_variants/$v/libmarlsched.so"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$O/$v" -o run -- \
    python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 1 --no-cpu-baseline > "$O/$v.json" 2> "$O/$v.err"
  echo "== $v"
  python3 "$R/profiles/summarize.py" "$O/$v"/run_kernel_stats.csv | grep -E "$RX"
  rm -f "$O/$v"/run_kernel_trace.csv
done
