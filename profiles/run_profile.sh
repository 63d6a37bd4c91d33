#!/usr/bin/env bash
# Profile the bench on a GPU box: kernel trace + stats, then separate PMC passes
# (FETCH_SIZE / WRITE_SIZE, one counter block per pass) for the env-step kernel.
# Usage (via gpurun): bash profiles/run_profile.sh <tag> [cfg2|cfg3|cfg4] (default cfg3, the headline)
set -euo pipefail
TAG="${1:-r1}"
CFG="${2:-cfg3}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/prof_${TAG}${2:+_$CFG}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
  python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 1 --no-cpu-baseline --no-step-kernel > "$OUT/bench.json" 2> "$OUT/trace.err"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_env_step|k_env_rollout_act_free' -f csv -d "$OUT/pmc_fetch" -o run -- \
  python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --update-step 20 --no-cpu-baseline --no-step-kernel > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_env_step|k_env_rollout_act_free' -f csv -d "$OUT/pmc_write" -o run -- \
  python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --update-step 20 --no-cpu-baseline --no-step-kernel > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
ALG=$(python3 -c "import json; r = json.load(open('$OUT/pmc_fetch.json'))['roofline']; print(r['bytes_per_env_round'] * r['envs_per_launch'])")
VAR=$(python3 -c "import json; r = json.load(open('$OUT/pmc_fetch.json'))['roofline']; print(r['variant'] if 'variant' in r else ('compact' if r.get('acceptor_observations', '').startswith('compact') else ''))")
KER=$(python3 -c "import json; r = json.load(open('$OUT/pmc_fetch.json'))['roofline']; print(r['kernel'].split('::')[-1])")
ROUNDS=1
[[ "$KER" == k_env_rollout_act_free ]] && ROUNDS=20  # (the PMC passes' --update-step)
python3 "$R/profiles/traffic_from_pmc.py" "$OUT/pmc_fetch/run_counter_collection.csv" "$OUT/pmc_write/run_counter_collection.csv" "$ALG" "$OUT/traffic.json" "$VAR" "$KER" "$ROUNDS"
echo "profile done: $OUT"
