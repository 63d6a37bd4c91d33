"""Profiling helper (not product): static instruction mix of one kernel's basic blocks from a hipcc -S
listing built with -gline-tables-only, each block tagged with the source lines it came from.
Usage: python tools/isa_blocks.py <file.s> <kernel symbol substring>"""
import re
import sys
from collections import Counter, defaultdict

path, sym = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
files = {}
for ln in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
start = next(i for i, ln in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(sym), ln))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
blocks, cur, name = [], None, "entry"
loc = None


def kind(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


cur = dict(name="entry", cnt=Counter(), src=Counter(), succ=[])
for ln in lines[start + 1:end]:
    s = ln.strip()
    if not s or s.startswith(";"):
        continue
    m = re.match(r"^(\.LBB\S+):", s)
    if m:
        blocks.append(cur)
        cur = dict(name=m.group(1), cnt=Counter(), src=Counter(), succ=[])
        continue
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
    if m:
        loc = "%s:%s" % (files.get(m.group(1), m.group(1)), m.group(2))
        continue
    if s.startswith("."):
        continue
    op = s.split()[0]
    k = kind(op)
    cur["cnt"][k] += 1
    if op in ("v_exp_f32", "v_rcp_f32", "v_log_f32", "v_mul_hi_u32", "v_mul_lo_u32", "v_sqrt_f32"):
        cur["cnt"]["slow:" + op] += 1
    if k in ("valu", "mfma") and loc:
        cur["src"][loc] += 1
    if op.startswith("s_cbranch") or op == "s_branch":
        cur["succ"].append(s.split()[-1])
blocks.append(cur)
tot = Counter()
for b in blocks:
    tot.update(b["cnt"])
    top = ", ".join("%s(%d)" % kv for kv in b["src"].most_common(4))
    c = b["cnt"]
    print("%-12s valu %4d mfma %3d salu %4d lds %3d vmem %3d  -> %-28s %s" % (
        b["name"], c["valu"], c["mfma"], c["salu"], c["lds"], c["vmem"], ",".join(b["succ"]), top))
print("total", dict(tot))
