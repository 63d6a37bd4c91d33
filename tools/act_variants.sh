#!/usr/bin/env bash
# tools/act_cost.py under library variants (tools/_variants/<name>/libmarlsched.so) and the in-tree
# library, on one box (via gpurun). Usage: bash tools/act_variants.sh <tag> "<variant names>"
set -euo pipefail
export MARLSCHED_LENIENT_ABI=1  # variants built at an older ABI load without the newer entry points
TAG="$1"; VARS="$2"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
for v in $VARS; do
  MARLSCHED_LIB="$R/tools/_variants/$v/libmarlsched.so" timeout -k 10 200 python tools/act_cost.py > "$O/act_$v.txt" 2>&1
  echo "== $v"; grep -v amdgpu.ids "$O/act_$v.txt"
done
timeout -k 10 200 python tools/act_cost.py > "$O/act_new.txt" 2>&1
echo "== new"; grep -v amdgpu.ids "$O/act_new.txt"
