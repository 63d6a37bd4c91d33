#!/usr/bin/env bash
# A/B of the env round (via gpurun): env GPU tests on the in-tree library, then alternating bench lines
# of tools/_variants/base (the previous library) and the in-tree one, then the phase probe.
# Usage: bash tools/ab_env.sh <tag> [pytest -k expression] ["base variant names", default base]
set -euo pipefail
TAG="$1"; K="${2:-env}"; BASE="${3:-base}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "$K" > "$O/tests.log" 2>&1
for i in 1 2; do
  for b in $BASE; do
    MARLSCHED_LIB="$R/tools/_variants/$b/libmarlsched.so" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 \
      > "$O/$b$i.json" 2> "$O/$b$i.err"
  done
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 > "$O/new$i.json" 2> "$O/new$i.err"
done
timeout -k 10 300 python tools/env_phase_probe.py > "$O/phase.txt" 2>&1
echo "ab done: $O"
