"""Per-kernel register / spill / occupancy table from hipcc's -Rpass-analysis=kernel-resource-usage
remarks. Usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kernel_resources.py [filter]"""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: (?:.*?)\s(Name|VGPRs|AGPRs|SGPRs|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill|"
                  r"ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" [")[0]] = v
flt = sys.argv[1] if len(sys.argv) > 1 else ""
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
except OSError:
    dem = names
for r, d in zip(rows, dem):
    if flt in d:
        print("%-60s vgpr %4s agpr %3s sgpr %4s occ %2s spillS %4s spillV %4s scratch %4s" % (
            d[:60], r.get("VGPRs"), r.get("AGPRs"), r.get("SGPRs"), r.get("Occupancy"), r.get("SGPRs Spill"),
            r.get("VGPRs Spill"), r.get("ScratchSize")))
