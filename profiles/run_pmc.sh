#!/usr/bin/env bash
# SQ instruction/wait counters for the hot kernels (separate pass, kernel-trace only).
# Usage (via gpurun): bash profiles/run_pmc.sh <tag>
set -euo pipefail
TAG="${1:-pmc}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_${TAG}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  --kernel-include-regex "k_env_step|k_act|k_ppo_grad" -f csv -d "$OUT/a" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --update-step 20 --no-cpu-baseline --no-graph > "$OUT/a.json" 2> "$OUT/a.err"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT \
  --kernel-include-regex "k_env_step|k_act|k_ppo_grad" -f csv -d "$OUT/b" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --update-step 20 --no-cpu-baseline --no-graph > "$OUT/b.json" 2> "$OUT/b.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE \
  --kernel-include-regex "k_env_step|k_act|k_ppo_grad|k_unit_returns" -f csv -d "$OUT/c" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --update-step 20 --no-cpu-baseline --no-graph > "$OUT/c.json" 2> "$OUT/c.err"
python3 "$R/profiles/pmc_summary.py" "$OUT/a/run_counter_collection.csv" "$OUT/b/run_counter_collection.csv" "$OUT/c/run_counter_collection.csv" | tee "$OUT/summary.txt"
