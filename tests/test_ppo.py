"""Host-side PPO logic on CPU: reference-order initialisation and the grouped
update against one reference PPO object per group (PPOmodules.py:75-174)."""
import numpy as np
import pytest
import torch

from oracle.ppo_ref import RefPPO


def _ppo_mod(ms):
    import importlib

    return importlib.import_module("marl-scheduling_amd.ppo")


def test_grouped_init_follows_reference_construction_order(ms):
    ppo = _ppo_mod(ms)
    torch.manual_seed(1234)
    refs = [RefPPO(11, 5, 0.003, 0.01, 0.9, 0.2, 3) for _ in range(4)]
    torch.manual_seed(1234)
    g = ppo.GroupedActorCritic(4, 11, 5)
    for i, r in enumerate(refs):
        for k, v in r.policy.flat().items():
            assert torch.equal(getattr(g, k)[i], v.detach()), k


@pytest.mark.parametrize("G,T,D,A,K", [(3, 50, 11, 5, 3), (2, 200, 18, 9, 1), (1, 64, 4, 13, 2)])
def test_grouped_update_matches_per_net_reference(ms, G, T, D, A, K):
    ppo = _ppo_mod(ms)
    torch.manual_seed(7)
    refs = [RefPPO(D, A, 0.003, 0.01, 0.87, 0.2, K) for _ in range(G)]
    torch.manual_seed(7)
    grp = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.87, 0.2, K, device="cpu")
    gen = torch.Generator().manual_seed(3)
    states = torch.randint(-5, 13, (G, T, D), generator=gen).float()
    actions = torch.randint(0, A, (G, T), generator=gen)
    old_lp = -torch.rand((G, T), generator=gen) * 3
    rewards = torch.randint(-6, 13, (G, T), generator=gen)
    rets = torch.stack([refs[g].returns(rewards[g].tolist()) for g in range(G)])
    ref_losses = [refs[g].update(states[g], actions[g], old_lp[g], rets[g]) for g in range(G)]
    losses = grp.update(states, actions, old_lp, rets)
    got = torch.stack(losses).T  # [G, K]
    np.testing.assert_allclose(got.numpy(), np.array(ref_losses), rtol=1e-5, atol=1e-6)
    for g in range(G):
        for k, v in refs[g].policy.flat().items():
            np.testing.assert_allclose(getattr(grp.policy, k)[g].detach().numpy(), v.detach().numpy(),
                                       rtol=1e-5, atol=1e-6, err_msg=k)


def test_k_epochs_rule():
    import importlib

    tr = importlib.import_module("marl-scheduling_amd.trainer")
    # trainPPO.py:76-77 with Python's half-even round; README.md:70-71 table
    assert tr._k_epochs(3, 1) == 3
    assert tr._k_epochs(3, 2) == 2   # round(1.5) = 2 (2-agent local sharing, ACCEPTOR_K 2)
    assert tr._k_epochs(3, 4) == 1   # round(0.75) = 1
    assert tr._k_epochs(3, 3) == 1
    assert tr._k_epochs(2, 8) == 1   # round(0.25) = 0 -> max(., 1)
    assert tr._k_epochs(5, 2) == 2   # round(2.5) = 2 (half-even)
