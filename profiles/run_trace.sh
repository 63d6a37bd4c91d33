#!/usr/bin/env bash
# Kernel trace + stats of one bench step (via gpurun): bash profiles/run_trace.sh <tag> [bench args]
set -euo pipefail
TAG="${1:-trace}"; shift || true
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/prof_${TAG}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/trace.err"
python3 "$R/profiles/summarize.py" "$OUT/run_kernel_stats.csv" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
