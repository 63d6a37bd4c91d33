"""Profiling helper: after one rollout, the price chooser's rows per update group (distinct 4-byte
rows, byte range) — what decides whether ms_ppo_grad's keyed path takes the group (<= 4096 distinct
rows, bytes in [-8, 24)). Usage: python tools/price_keys_probe.py [rollout_streams]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
streams = int(sys.argv[1]) if len(sys.argv) > 1 else 1
tr = tr_mod.Trainer.from_named("cfg3", rollout_streams=streams, device="cuda:0")
tr.rollout()
torch.cuda.synchronize()
po = tr.price_obs[: tr.T]  # [T][E][U][4]
L = tr.L
for a in range(tr.N):
    for l in (0, L - 1):
        u = a * L + l
        rows = po[:, :, u, :].reshape(-1, 4)
        w = rows.contiguous().view(torch.int32).view(-1)
        n = torch.unique(w).numel()
        print("streams %d unit %2d: rows %d distinct %d bytes [%d, %d]" % (streams, u, w.numel(), n, int(rows.min()),
                                                                             int(rows.max())))
