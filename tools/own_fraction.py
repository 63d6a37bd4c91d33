"""Fraction of cfg5 agent rows whose agent owns no core (acceptor layer 1 = base exactly), over frames."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

importlib.import_module("marl-scheduling_amd")
bdqn = importlib.import_module("marl-scheduling_amd.bdqn")
abi = importlib.import_module("marl-scheduling_amd.abi")
tr = bdqn.BDQNTrainer(abi.named_config("cfg5"), n_envs=2048, bcfg=bdqn.BDQNConfig(memory_frames=8, learning_starts=4),
                      seed=0, device=torch.device("cuda", 0))
for f in range(60):
    tr.step()
    if f % 10 == 9:
        own = tr.core_owner[tr.head].long()  # [E, C], 0 = free, a + 1 = agent a
        E, C = own.shape
        N = tr.N
        owns = torch.zeros((E, N + 1), dtype=torch.int64, device=own.device)
        owns.scatter_add_(1, own, torch.ones_like(own))
        none = (owns[:, 1:] == 0).float().mean().item()
        print("frame %d: agents owning no core %.3f, free cores %.3f" % (f + 1, none, (own == 0).float().mean().item()),
              flush=True)
