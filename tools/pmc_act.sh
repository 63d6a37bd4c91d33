#!/usr/bin/env bash
# PMC instruction / wait counters of the act kernels, each launched on its own by tools/act_cost.py
# (core chooser, core + price chooser, compact acceptors, the paired launch). Via gpurun.
set -euo pipefail
TAG="$1"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
pass() {
  local name="$1"; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "k_act" -f csv -d "$OUT/$name" -o run -- \
    python3 "$R/tools/act_cost.py" > "$OUT/$name.txt" 2> "$OUT/$name.err"
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
pass b SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR
python3 "$R/profiles/pmc_summary.py" "$OUT"/{a,b}/run_counter_collection.csv > "$OUT/summary.txt"
rm -rf "$OUT/a" "$OUT/b"
echo "pmc_act done"
