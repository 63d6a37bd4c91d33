"""Where the waves of the one-launch cfg3 rollout (k_env_rollout_act_free) spend a round (profiling only).

Loads the probe build (tools/_probe/libmarlsched_probe.so from tools/build_phase_probe.sh, -DMS_PHASE_TIMING)
in place of the product library, runs cfg3 PPO iterations (one rollout launch each), and prints per wave and
round the shader cycles of its five phases: the env round (k_env_step's round of its 4 replicas), the wait at
the workgroup barrier after it, its agent's offer units, its agent's acceptors, and the wait at the barrier after
that. Large waits mean
the workgroup's waves are unbalanced (the slowest wave of a phase holds the other seven)."""
import ctypes as ct
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["MARLSCHED_LIB"] = os.path.join(ROOT, "tools", "_probe", "libmarlsched_probe.so")
os.environ["MARLSCHED_LENIENT_ABI"] = "1"


def main(E=16384, iters=3, T=200):
    import torch
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    lib_mod = importlib.import_module("marl-scheduling_amd._lib")
    lib = lib_mod.lib
    lib.ms_probe_free_cycles.argtypes = [ct.POINTER(ct.c_ulonglong), ct.c_int, ct.c_int]
    tr = tr_mod.Trainer.from_named("cfg3", n_envs=E, update_step=T, seed=0, device="cuda:0")
    assert tr.fused_rollout_free
    waves = E // 4
    buf = (ct.c_ulonglong * (5 * waves))()
    names = ("env round", "wait after env", "offer units", "acceptors", "wait after acting")
    for it in range(iters):
        tr.rollout()
        torch.cuda.synchronize()
        assert lib.ms_probe_free_cycles(buf, waves, 1) == 0
        tr.update()
        torch.cuda.synchronize()
        if it == 0:
            continue  # the first rollout runs eagerly before its graph capture: two launches' worth
        c = np.frombuffer(buf, dtype=np.uint64).reshape(waves, 5).astype(np.float64) / T
        tot = c.sum(1)
        print("iteration %d: cycles per wave per round (mean / p10 / p50 / p90 over %d waves)" % (it, waves))
        for k, n in enumerate(names):
            v = c[:, k]
            print("  %-18s %8.0f %8.0f %8.0f %8.0f  (%4.1f %%)" % (n, v.mean(), np.percentile(v, 10),
                                                                 np.percentile(v, 50), np.percentile(v, 90),
                                                                 100 * v.mean() / tot.mean()))
        print("  %-18s %8.0f" % ("total", tot.mean()))
        # per agent (wave index within the workgroup) acting cycles
        for k, n in ((2, "offers"), (3, "acceptors")):
            ag = c[:, k].reshape(-1, 8).mean(0)
            print("  %-10s by agent: " % n + " ".join("%.0f" % x for x in ag))
    print("clock: the bench's clock_mhz converts cycles to us")


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
