"""Profiling helper (not product): fraction of acceptor rows equal to the common row after a short
rollout of the cfg3 trainer, and the act kernel's time with and without the common-row path."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ms = importlib.import_module("marl-scheduling_amd")
tr_mod = importlib.import_module("marl-scheduling_amd.trainer")

tr = tr_mod.Trainer.from_named("cfg3", n_envs=int(os.environ.get("E", 16384)), update_step=50, seed=1, device="cuda:0")
tr.iteration()
torch.cuda.synchronize()
obs = tr.acceptor_rows(10, 11)[0].contiguous()
crow = tr.acc_common
eq = (obs == crow).all(-1)
print("common fraction", eq.float().mean().item(), "per agent-core:", eq.float().mean(0).view(8, 8).mean(1).tolist())
net = tr.acc.group.policy_old
U = obs.shape[1]
for common in (None, crow):
    for _ in range(3):
        net.act(obs, U, 1, 2, common_row=common)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        net.act(obs, U, 1, 2, common_row=common)
    e.record()
    torch.cuda.synchronize()
    print("common" if common is not None else "plain", "us per act", s.elapsed_time(e) / 20 * 1000)
