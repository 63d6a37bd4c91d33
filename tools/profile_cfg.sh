#!/usr/bin/env bash
# Kernel trace + stats of the other BASELINE workloads' bench lines (via gpurun).
# Usage: bash tools/profile_cfg.sh <tag> [configs...]   (default: cfg4 cfg5)
set -euo pipefail
TAG="$1"; shift
CFGS=("$@"); [[ ${#CFGS[@]} -eq 0 ]] && CFGS=(cfg4 cfg5)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
for c in "${CFGS[@]}"; do
  cd "$R"
  timeout -k 10 300 python bench.py --config "$c" --no-cpu-baseline > "$O/$c.json" 2> "$O/$c.err"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace_$c" -o run -- \
    python3 "$R/bench.py" --config "$c" --steps 1 --warmup 1 --no-cpu-baseline > "$O/trace_$c.json" 2> "$O/trace_$c.err"
  python3 "$R/profiles/summarize.py" "$O/trace_$c/run_kernel_stats.csv" > "$O/kernel_summary_$c.txt"
  cp "$O/trace_$c/run_kernel_stats.csv" "$O/kernel_stats_$c.csv"
  rm -rf "$O/trace_$c"   # the per-dispatch trace is tens of MB (gpurun_out returns at most 64 MiB)
done
echo "profile_cfg done: $O"
