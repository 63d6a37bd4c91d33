"""Per-wave timing of the compact acceptor gradient (k_ppo_grad<.., kOwnerRow>) at cfg3: entry, end of
the scan + listed-row tiles, exit (s_memrealtime, 100 MHz) and the rows each wave listed for its tiles.
Needs the probe build: bash tools/build_variant.sh gprobe -DMS_GRAD_PROBE, then
MARLSCHED_LIB=tools/_variants/gprobe/libmarlsched.so python tools/grad_probe.py (profiling only)."""
import ctypes as ct
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
importlib.import_module("marl-scheduling_amd")
trainer_mod = importlib.import_module("marl-scheduling_amd.trainer")
lib_mod = importlib.import_module("marl-scheduling_amd._lib")

tr = trainer_mod.Trainer.from_named(os.environ.get("CFG", "cfg3"), n_envs=int(os.environ.get("E", "16384")), update_step=200, seed=0,
                                    device=torch.device("cuda:0"))
for _ in range(2):
    tr.iteration()
torch.cuda.synchronize()
NW = 1 << 15
buf = np.zeros((NW, 4), dtype=np.uint64)
lib = lib_mod.lib if hasattr(lib_mod, "lib") else lib_mod.load()
rc = lib.ms_grad_probe_read(buf.ctypes.data_as(ct.c_void_p), ct.c_size_t(buf.nbytes))
assert rc == 0, rc
used = buf[:, 2] > 0
b = buf[used]
t0 = b[:, 0].astype(np.int64)
base = t0.min()
start = (t0 - base) / 100.0  # us
scan = (b[:, 1].astype(np.int64) - t0) / 100.0
life = (b[:, 2].astype(np.int64) - t0) / 100.0
end = (b[:, 2].astype(np.int64) - base) / 100.0
listed = (b[:, 3] & 0xffffffff).astype(np.int64)
grp = (b[:, 3] >> 32).astype(np.int64)
pct = [0, 10, 50, 90, 99, 100]
print("waves", used.sum(), "launch span %.1f us" % end.max(), "scan-only waves (none listed): lifetime mean %.1f us" % life[listed == 0].mean() if (listed == 0).any() else "")
for name, v in (("start", start), ("scan+tiles", scan), ("lifetime", life), ("end", end), ("listed", listed)):
    print("%-11s" % name, " ".join("%9.1f" % np.percentile(v, q) for q in pct))
for g in range(min(grp.max() + 1, 16)):
    m = grp == g
    print("group %d: waves %d listed mean %.0f max %d lifetime mean %.1f max %.1f us" % (
        g, m.sum(), listed[m].mean(), listed[m].max(), life[m].mean(), life[m].max()))
