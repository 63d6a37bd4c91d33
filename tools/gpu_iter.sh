#!/usr/bin/env bash
# One GPU iteration (via gpurun): selected GPU tests, the bench line, and a kernel trace of one bench
# step. Usage: bash tools/gpu_iter.sh <tag> [pytest -k expression] [extra bench args]
set -euo pipefail
TAG="$1"; K="${2:-}"; shift 2 || true
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
if [[ -n "$K" ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "$K" > "$O/tests.log" 2>&1
fi
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$O/bench.json" 2> "$O/bench.err"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline "$@" > "$O/trace_bench.json" 2> "$O/trace.err"
python3 "$R/profiles/summarize.py" "$O/trace/run_kernel_stats.csv" > "$O/kernel_summary.txt"
echo "gpu_iter done: $O"
