#!/usr/bin/env bash
# Launch-shape sweep of the paired act kernel (MS_ACT_PAIR_WAVES, MS_ACT_PAIR_COMMON_WAVES) on the cfg3 bench.
# Usage (via gpurun): bash tools/sweep_act.sh <tag>
set -euo pipefail
TAG="${1:-sweep}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
IFS=, read -ra CFGS <<< "${MS_SWEEP:-2048 768,1024 768,1536 768,3072 768,768 768}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  MS_ACT_PAIR_WAVES=$1 MS_ACT_PAIR_COMMON_WAVES=$2 timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline \
    > "$O/b_$1_$2.json" 2> "$O/b_$1_$2.err"
  python3 -c "import json,sys; d=json.load(open('$O/b_$1_$2.json')); print('$1 $2', round(d['ms_per_step'],3), {k: round(v,3) if isinstance(v,float) else v for k,v in d['breakdown_ms_per_step'].items()})" | tee -a "$O/summary.txt"
done
