#!/usr/bin/env bash
# A/B of a library variant against the in-tree library (via gpurun): the env GPU tests on the variant,
# alternating bench lines (in-tree, variant) x 2, then the PMC passes of the variant's bench.
# Usage: bash tools/ab_variant.sh <tag> <variant dir under tools/_variants> [pytest -k expr] [bench args]
set -euo pipefail
TAG="$1"; V="$2"; K="${3:-env or kats or configs}"; shift 3 || shift $#
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
VL="$R/tools/_variants/$V/libmarlsched.so"
mkdir -p "$O"
cd "$R"
MARLSCHED_LIB="$VL" timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "$K" > "$O/tests.log" 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 "$@" > "$O/base$i.json" 2> "$O/base$i.err"
  MARLSCHED_LIB="$VL" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 "$@" > "$O/new$i.json" 2> "$O/new$i.err"
done
MARLSCHED_LIB="$VL" bash profiles/run_pmc.sh "$TAG" > "$O/pmc.log" 2>&1
echo "ab done: $O"
