#!/usr/bin/env bash
# Round-end style GPU check (via gpurun): the whole -m gpu suite, smoke(), the rocprof profile of the
# bench (kernel trace + env-step PMC traffic), the default bench line and the other configs' lines.
# Usage: bash tools/round_check.sh <tag>
set -euo pipefail
TAG="$1"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$O/gputest.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
bash profiles/run_profile.sh "$TAG" > "$O/profile.log" 2>&1
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config "$c" --no-cpu-baseline > "$O/$c.json" 2> "$O/$c.err"
done
echo "round check done: $O"
