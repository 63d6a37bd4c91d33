#!/usr/bin/env bash
# Kernel trace of a few cfg5 frames (via gpurun), the per-dispatch CSV kept small: frames 30..34 only.
set -euo pipefail
TAG="$1"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$O/trace5" -o run -- \
  python3 "$R/bench.py" --config cfg5 --steps 1 --warmup 0 --update-step 40 --no-cpu-baseline > "$O/trace5.json" 2> "$O/trace5.err"
python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
f = glob.glob(o + "/trace5/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
env = [i for i, r in enumerate(rows) if "k_env_step" in r["Kernel_Name"]]
a, b = env[30], env[34]   # four frames, from one env step to the fourth after it
span = rows[a:b]
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in span:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = r["Kernel_Name"][:90]
    tot[k] += d; cnt[k] += 1
wall = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3 / 4
busy = sum(tot.values()) / 4
with open(o + "/frame_breakdown.txt", "w") as out:
    out.write("per frame: wall %.1f us, kernel busy %.1f us, %d dispatches\n" % (wall, busy, len(span) / 4))
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:40]:
        out.write("%-90s %5.1f calls %9.1f us/frame\n" % (k, cnt[k] / 4, v / 4))
    # idle gaps between consecutive dispatches (device idle: the host had not queued the next one)
    gaps = collections.defaultdict(float)
    for p_, n_ in zip(span, span[1:]):
        g = (int(n_["Start_Timestamp"]) - int(p_["End_Timestamp"])) / 1e3
        if g > 0:
            gaps[(p_["Kernel_Name"][:50], n_["Kernel_Name"][:50])] += g
    out.write("\nidle gaps per frame (previous -> next dispatch):\n")
    for (a_, b_), g in sorted(gaps.items(), key=lambda x: -x[1])[:15]:
        out.write("%8.1f us  %s  ->  %s\n" % (g / 4, a_, b_))
PY
rm -rf "$O/trace5"
echo "trace_cfg5 done"
