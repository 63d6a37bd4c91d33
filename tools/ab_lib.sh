#!/usr/bin/env bash
# Alternating cfg3 bench lines of library variants (tools/_variants/<name>/libmarlsched.so) and the in-tree
# library on one box (via gpurun). Usage: bash tools/ab_lib.sh <tag> "<variant names>" [rounds]
set -euo pipefail
TAG="$1"; VARS="$2"; N="${3:-2}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
for i in $(seq 1 "$N"); do
  for v in $VARS; do
    MARLSCHED_LIB="$R/tools/_variants/$v/libmarlsched.so" timeout -k 10 300 python bench.py --no-cpu-baseline \
      --no-step-kernel --steps 8 > "$O/$v$i.json" 2> "$O/$v$i.err"
  done
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-step-kernel --steps 8 > "$O/new$i.json" 2> "$O/new$i.err"
done
python3 - "$O" <<'PY'
import glob, json, os, sys
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    d = json.load(open(f))
    r = d["roofline"]
    print("%-12s %8.3f ms  env %6.2f us  frac %.3f  rollout %.3f update %.3f" % (
        os.path.basename(f)[:-5], d["ms_per_step"], r["avg_launch_us"], r["frac"],
        d["breakdown_ms_per_step"]["rollout"], d["breakdown_ms_per_step"]["update"]))
PY
echo "ab_lib done: $O"
