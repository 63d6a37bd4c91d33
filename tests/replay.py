"""Trainer rings replayed through the C oracle (test infrastructure): the observations and rewards a
trainer's rollout rings hold for sampled replicas against oracle/ms_oracle.c stepped with the actions
the same rings hold (world.py:295-334, Reward.py)."""
import importlib

import numpy as np
import torch

from oracle import pyoracle


def _ppo():
    return importlib.import_module("marl-scheduling_amd.ppo")


def oracle_replay(tr, replicas, base_seed, T):
    """Step the C oracle of replicas e with the actions the trainer's rings hold and compare its
    observations and rewards with the rings (slot t + 1 = the observation after round t)."""
    cfg = tr.cfg
    s = pyoracle.abi.config_shape(cfg)
    N, C, L, D_acc, D_off = s["N"], s["C"], s["L"], s["acc_obs_dim"], s["off_obs_dim"]
    idx = torch.tensor(list(replicas), device=tr.acc_rows.device)
    acc_all = _ppo().regen_acceptor_rows(tr.acc_rows.index_select(1, idx).contiguous(),
                                         tr.acc_owner.index_select(1, idx).contiguous(), tr.acc_common,
                                         tr.N).cpu().numpy()                # [T+1, n, N*C, stride]
    off_all = tr.off_obs[:, list(replicas)].cpu().numpy()
    aa = tr.acc.actions[:, list(replicas)].cpu().numpy()
    ao = tr.off.actions[:, list(replicas)].cpu().numpy()
    ap = tr.price.actions[:, list(replicas)].cpu().numpy() if tr.free else None
    ra = tr.acc.rewards[:, list(replicas)].cpu().numpy()
    ro = tr.off.rewards[:, list(replicas)].cpu().numpy()
    rp = tr.price.rewards[:, list(replicas)].cpu().numpy() if tr.free else None
    for i, e in enumerate(replicas):
        env = pyoracle.OracleEnv(cfg, base_seed + e)
        o = env.observe()
        assert np.array_equal(acc_all[0, i, :, :D_acc].reshape(N, C, D_acc), o["acceptor"]), e
        for t in range(T):
            core = ao[t, i].reshape(N, L)
            price = np.where(core == 0, -5, ap[t, i].reshape(N, L)) if tr.free else None
            r = env.step(aa[t, i].reshape(N, C), core, price)
            o = env.observe()
            assert np.array_equal(acc_all[t + 1, i, :, :D_acc].reshape(N, C, D_acc), o["acceptor"]), (e, t)
            assert np.array_equal(off_all[t + 1, i, :, :D_off].reshape(N, L, D_off), o["offer"]), (e, t)
            assert np.array_equal(ra[t, i].reshape(N, C), r["acceptor"]), (e, t)
            assert np.array_equal(ro[t, i].reshape(N, L), r["offer"]), (e, t)
            if tr.free:
                assert np.array_equal(rp[t, i].reshape(N, L), r["price"]), (e, t)
