#!/usr/bin/env bash
# SQ instruction/wait counters and memory-side request counters for the hot kernels, each
# counter group in its own pass (kernel-trace only). Usage (via gpurun):
#   bash profiles/run_pmc.sh <tag> [cfg2|cfg3|cfg4] [kernel regex]
set -euo pipefail
TAG="${1:-pmc}"
CFG="${2:-cfg3}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_${TAG}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
KR="${3:-k_env_step|k_act|k_ppo_grad|k_unit_returns|k_key|k_own}"
pass() {  # pass <name> <counters...>
  local name="$1"; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$KR" -f csv -d "$OUT/$name" -o run -- \
    python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --update-step 20 --no-cpu-baseline --no-graph \
    --no-step-kernel > "$OUT/$name.json" 2> "$OUT/$name.err"
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
pass b SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR
pass c TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_64B_sum
pass d FETCH_SIZE
pass e WRITE_SIZE
python3 "$R/profiles/pmc_summary.py" "$OUT"/{a,b,c,d,e}/run_counter_collection.csv | tee "$OUT/summary.txt"
