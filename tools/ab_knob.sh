#!/usr/bin/env bash
# Alternating cfg3 bench lines with an environment knob set (A) and unset (B) on one box (via gpurun).
# Usage: bash tools/ab_knob.sh <tag> "<VAR=value ...>" [rounds]
set -euo pipefail
export MARLSCHED_LENIENT_ABI=1  # variants built at an older ABI load without the newer entry points
TAG="$1"; KNOB="$2"; N="${3:-2}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
for i in $(seq 1 "$N"); do
  env $KNOB timeout -k 10 300 python bench.py --no-cpu-baseline --no-step-kernel --steps 8 > "$O/knob$i.json" 2> "$O/knob$i.err"
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
echo "ab_knob done: $O"
