"""Cycle attribution of k_env_step phases (profiling only; uses tools/_probe/libmarlsched_probe.so
built by tools/build_phase_probe.sh, never the product library's code path).

Runs cfg3 at E replicas with random actions and prints, per phase mark, the average cycles one
wave spends between the previous mark and this one (lane 0's s_memtime deltas)."""
import ctypes as ct
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
abi = importlib.import_module("marl-scheduling_amd.abi")
NAMES = {1: "stage (+ successor MT twist)", 2: "MT peek + masks + liab prefetch", 3: "auctioneer + spawn peek",
         4: "exec select + rank", 5: "executions", 6: "tick + settlement", 7: "offers", 8: "spawn",
         9: "record round/mti", 10: "write record + rewards", 11: "rebuild masks", 12: "emit observations"}
ORDER = list(range(1, 13))


def main(E=16384, steps=20, min_lpe=None, compact=True):
    d = "_probe" + ("_lpe%d" % min_lpe if min_lpe else "")
    lib = ct.CDLL(os.path.join(ROOT, "tools", d, "libmarlsched_probe.so"))
    lib.ms_env_create.argtypes = [ct.POINTER(abi.MsConfig), ct.c_int64, ct.c_uint64, ct.POINTER(ct.c_void_p)]
    lib.ms_env_step.argtypes = [ct.c_void_p, ct.POINTER(abi.MsActions), ct.POINTER(abi.MsObsOut),
                                ct.POINTER(abi.MsRewardOut), ct.c_void_p, ct.c_void_p]
    lib.ms_env_shape.argtypes = [ct.c_void_p, ct.POINTER(abi.MsShape)]
    lib.ms_probe_phase_cycles.argtypes = [ct.POINTER(ct.c_ulonglong), ct.c_int]
    cfg = abi.named_config("cfg3")
    h = ct.c_void_p()
    assert lib.ms_env_create(ct.byref(cfg), E, 0, ct.byref(h)) == 0
    sh = abi.MsShape()
    lib.ms_env_shape(h, ct.byref(sh))
    N, C, L, O = sh.n_agents, sh.n_cores, sh.collection_length, sh.max_offers
    d = torch.device("cuda")
    g = torch.Generator(device=d).manual_seed(0)
    acc = torch.randint(0, O + 1, (steps + 5, E, N, C), device=d, generator=g, dtype=torch.int32).to(torch.int8)
    off = torch.randint(0, C + 1, (steps + 5, E, N, L), device=d, generator=g, dtype=torch.int32).to(torch.int8)
    price = torch.randint(0, 13, (steps + 5, E, N, L), device=d, generator=g, dtype=torch.int32).to(torch.int8)
    oa = torch.empty((E, N, C, sh.acc_obs_stride), dtype=torch.int8, device=d)
    oo = torch.empty((E, N, L, sh.off_obs_stride), dtype=torch.int8, device=d)
    rw = [torch.empty((E, N, L), device=d), torch.empty((E, N, L), device=d),
          torch.empty((E, N, C), dtype=torch.int32, device=d), torch.empty((E, C), dtype=torch.int32, device=d),
          torch.empty((E, N), dtype=torch.int32, device=d)]
    if compact:  # the training round's form: owner row per core + the owners (k_env_step<LPE, false, true>)
        cr = torch.empty((E, C, sh.acc_obs_stride), dtype=torch.int8, device=d)
        co = torch.empty((E, C), dtype=torch.int8, device=d)
        obs = abi.MsObsOut(None, oo.data_ptr(), None, cr.data_ptr(), co.data_ptr())
    else:
        obs = abi.MsObsOut(oa.data_ptr(), oo.data_ptr(), None)
    rew = abi.MsRewardOut(*[t.data_ptr() for t in rw])
    buf = (ct.c_ulonglong * 16)()

    def run(t):
        a = abi.MsActions(acc[t].data_ptr(), off[t].data_ptr(), price[t].data_ptr(), None)
        st = ct.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert lib.ms_env_step(h, ct.byref(a), ct.byref(obs), ct.byref(rew), None, st) == 0

    for t in range(5):
        run(t)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()  # device time without host gaps between launches
    with torch.cuda.graph(graph):
        for t in range(steps):
            run(5 + t)
    torch.cuda.synchronize()
    lib.ms_probe_phase_cycles(buf, 1)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    graph.replay()
    ev[1].record()
    torch.cuda.synchronize()
    lib.ms_probe_phase_cycles(buf, 0)
    lpe = min_lpe or 16
    while lpe < max(N, C):
        lpe *= 2
    waves = (E + 64 // lpe - 1) // (64 // lpe)
    n_blocks = waves
    tot = sum(buf[k] for k in ORDER)
    print("k_env_step (probe build, %d lanes/env) %.1f us/step; per wave: %.0f cycles" % (lpe, ev[0].elapsed_time(ev[1]) * 1e3 / steps,
                                                                        tot / waves / steps))
    for k in ORDER:
        print("  %2d %-34s %8.0f cycles/wave  %5.1f%%" % (k, NAMES[k], buf[k] / waves / steps, 100.0 * buf[k] / tot))
    # entry / exit times of every wave of the last launch (s_memrealtime, 100 MHz)
    import numpy as np
    spans = (ct.c_ulonglong * (2 * n_blocks))()
    lib.ms_probe_wave_spans.argtypes = [ct.POINTER(ct.c_ulonglong), ct.c_int]
    assert lib.ms_probe_wave_spans(spans, n_blocks) == 0
    sp = np.array(spans[:], dtype=np.float64).reshape(n_blocks, 2) / 100.0  # us
    t0 = sp[:, 0].min()
    st, en, life = sp[:, 0] - t0, sp[:, 1] - t0, sp[:, 1] - sp[:, 0]
    q = [0, 10, 50, 90, 99, 100]
    fmt = lambda a: " ".join("%6.1f" % v for v in np.percentile(a, q))
    print("  wave spans of the last launch (us; percentiles %s):" % q)
    print("    entry    %s" % fmt(st))
    print("    exit     %s" % fmt(en))
    print("    lifetime %s" % fmt(life))
    # one more launch alone: every wave's phase cycles against its lifetime (where the slow waves
    # lose their time)
    lib.ms_probe_phase_cycles(buf, 1)
    run(4)
    torch.cuda.synchronize()
    lib.ms_probe_phase_blocks.argtypes = [ct.POINTER(ct.c_ulonglong), ct.c_int]
    pb = (ct.c_ulonglong * (16 * n_blocks))()
    assert lib.ms_probe_phase_blocks(pb, n_blocks) == 0
    assert lib.ms_probe_wave_spans(spans, n_blocks) == 0
    ph = np.array(pb[:], dtype=np.float64).reshape(n_blocks, 16)
    sp = np.array(spans[:], dtype=np.float64).reshape(n_blocks, 2) / 100.0
    life = sp[:, 1] - sp[:, 0]
    order = np.argsort(life)
    slow, mid = order[-max(1, n_blocks // 10):], order[n_blocks // 2 - n_blocks // 20: n_blocks // 2 + n_blocks // 20]
    print("  one launch: lifetime %s us; phase cycles per wave, median-lifetime waves vs slowest 10%%:" % fmt(life))
    for k in ORDER:
        print("  %2d %-34s %8.0f %8.0f  (p10 %6.0f p90 %6.0f)" % (k, NAMES[k], ph[mid, k].mean(), ph[slow, k].mean(),
                                                               np.percentile(ph[:, k], 10), np.percentile(ph[:, k], 90)))
    xcd = np.arange(n_blocks) % 8
    print("  mean lifetime per XCD (block %% 8): " + " ".join("%.1f" % life[xcd == x].mean() for x in range(8)))
    q4 = np.arange(n_blocks) * 4 // n_blocks
    print("  mean lifetime per grid quarter: " + " ".join("%.1f" % life[q4 == x].mean() for x in range(4)))


if __name__ == "__main__":
    main(min_lpe=int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1] != "0" else None,
         compact=not (len(sys.argv) > 2 and sys.argv[2] == "materialised"))
