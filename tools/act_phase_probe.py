"""Cycle attribution of the paired act kernel's phases (profiling only): the cfg3 trainer runs on the probe
library (tools/build_act_probe.sh; MARLSCHED_LIB points the package at it), and after its rollouts the
per-(half, phase) shader-clock cycles lane 0 of every wave accumulated are printed as cycles per wave.
Usage: MARLSCHED_LIB=tools/_probe_act/libmarlsched.so python tools/act_phase_probe.py [iterations]"""
import ctypes as ct
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
assert "_probe_act" in os.environ.get("MARLSCHED_LIB", ""), "run with MARLSCHED_LIB=tools/_probe_act*/libmarlsched.so"
_lib = importlib.import_module("marl-scheduling_amd._lib")
tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
lib = _lib.lib
lib.ms_probe_act_cycles.argtypes = [ct.POINTER(ct.c_ulonglong), ct.c_int]
NAMES = [
    {0: "setup (fragments, price digits, first loads)", 1: "row indices + next loads issued", 2: "Philox",
     3: "core chooser (layer 1 waits for rows)", 4: "price chooser (input, table, sample, stores)",
     5: "core chooser stores", 6: "untabulated price inputs"},
    {0: "setup (fragments, common table)", 1: "owner loads issued", 2: "scan bookkeeping", 3: "Philox",
     4: "table search, stores, row list", 5: "list + first tile loads", 6: "listed rows: layer 1",
     7: "listed rows: layers 2-3 + sample", 8: "listed rows: stores"},
]


def main(iters=2):
    tr = tr_mod.Trainer.from_named("cfg3", seed=1, device="cuda:0", use_graph=False)
    tr.iteration()  # warm
    torch.cuda.synchronize()
    buf = (ct.c_ulonglong * 34)()
    lib.ms_probe_act_cycles(buf, 1)
    for _ in range(iters):
        tr.rollout()
        tr.update()
    torch.cuda.synchronize()
    assert lib.ms_probe_act_cycles(buf, 1) == 0
    for half in range(2):
        row = [buf[17 * half + k] for k in range(17)]
        waves = row[16]
        tot = sum(row[:16]) / max(waves, 1)
        print("%s half: %d waves, %.0f cycles per wave" % (("offer", "acceptor")[half], waves, tot))
        for k, name in NAMES[half].items():
            c = row[k] / max(waves, 1)
            print("  %-48s %8.0f  %5.1f %%" % (name, c, 100.0 * c / max(tot, 1)))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2)
