"""The E = 1 drop-in DQN env (DQNDividedFixedPricesEnv, SchedulingEnvironment.py:351-436) driven by the
loop body of trainDQN.py:126-268, against the object-faithful world (oracle/pyref.py) with the
reference's DQN agents restated in torch fp32 on the same random streams (oracle/dqn_ref.py)."""
import random

import numpy as np
import pytest
import torch

from tests.test_dropin import _as_lists, _mods, _pyref_config, world_params


def dqn_params(batch=10, mem=40):
    return {"BATCH_SIZE": batch, "OFFER_GAMMA": 0.5, "ACCEPTOR_GAMMA": 0.84, "RUN_START": 0.9,
            "REPLAY_MEMORY_SIZE": mem, "RUN_END": 0.05, "RUN_DECAY": 30, "TARGET_UPDATE": 2,
            "RANDOMPOLICY": False, "IS_DQN": True, "freePrices": False, "netZeroOfferReward": 0.5}


def test_dqn_env_is_exported():
    _, env_mod, _ = _mods()
    assert hasattr(env_mod, "DQNDividedFixedPricesEnv") and hasattr(env_mod, "DQNSchedulingEnv")


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,L,mem", [(2, 2, 3, 40), (3, 2, 2, 25)])
def test_dropin_dqn_env_matches_reference_agents(N, C, L, mem):
    from oracle.dqn_ref import RefDQNAgents
    from oracle.pyref import PyWorld

    world, env_mod, _ = _mods()
    wp = world_params(N=N, C=C, L=L, ep=15)
    rp = dqn_params(mem=mem)
    seed = 99
    random.seed(seed)
    np.random.seed(5)
    torch.manual_seed(3)
    w = world.World(wp)
    env = env_mod.DQNDividedFixedPricesEnv(w, rp)
    # the reference's agents on the object-faithful world, same seeds
    pw = PyWorld(_pyref_config(wp, False), seed)
    torch.manual_seed(3)
    sh = env._eng.env.shape
    ref = RefDQNAgents(pw, dict(acc=(sh.acc_obs_dim, sh.acc_actions), off=(sh.off_obs_dim, sh.off_actions)), rp)
    n_greedy_checked = 0
    for i_episode in range(3):  # trainDQN.py:126-268
        newAcc, newOff, newAuct = env.reset()
        r_obs = pw.observe()
        for t in range(1000):
            acceptorActions, offerActions = env.getActionForAllAgents(newAcc, newOff)
            r_acc, r_off = ref.get_actions(r_obs[0], r_obs[1])  # same stream state: pw.rng == random
            assert acceptorActions == r_acc and offerActions == r_off, (i_episode, t)
            n_greedy_checked += sum(isinstance(v, int) for row in r_acc + r_off for v in row)
            assert pw.rng.getstate() == random.getstate()
            auctioneer_action = w.auctioneer.getAuctioneerAction(newAuct)
            assert pw.auctioneer_actions() == auctioneer_action
            env.oldAcceptorObservationTensors = newAcc
            env.oldOfferObservationTensors = newOff
            (newAcc, newOff, newAuct, offerRewards, acceptorRewards, auctioneerReward, agentReward, acceptionQuality,
             done) = env.step(offerActions, acceptorActions, auctioneer_action)
            old_r = r_obs
            # world.py:399 takes int(chosenIndexValue); :412-413 compares coreID == action + 1 (3.0 == 3)
            ints = lambda rows: [[int(v) for v in row] for row in rows]
            r_obs, r_rew, _, r_done = pw.step(ints(r_acc), ints(r_off), auctioneer_action)
            assert _as_lists(newAcc) == r_obs[0] and _as_lists(newOff) == r_obs[1] and done == r_done
            env.newAcceptorObservationTensors = newAcc
            env.newOfferObservationTensors = newOff
            if done:
                break
            np_before = np.random.get_state()
            env.updateAcceptorMemoriesAndOptimize(acceptorActions, acceptorRewards)
            env.updateOfferMemoriesAndOptimize(offerActions, offerRewards)
            np_dropin = np.random.get_state()
            np.random.set_state(np_before)
            ref.update("acc", r_acc, r_rew[1], old_r[0], r_obs[0], rp["ACCEPTOR_GAMMA"])
            ref.update("off", r_off, r_rew[0], old_r[1], r_obs[1], rp["OFFER_GAMMA"])
            assert np.array_equal(np_dropin[1], np.random.get_state()[1])  # the same minibatch draws
            assert random.getstate() == pw.rng.getstate()
        if (i_episode % rp["TARGET_UPDATE"]) == 0:
            for agent in w.agents:
                agent.updateTargetNets()
            for a in range(N):
                ref.update_targets(a)
    assert w.round == 45 and n_greedy_checked > 0
    dqn = env._dqn
    for kind in ("acc", "off"):
        g = env._groups[kind]
        for u, net in enumerate(ref.policy[kind]):
            for k, p in zip(dqn.KEYS, (net[0].weight, net[0].bias, net[2].weight, net[2].bias)):
                np.testing.assert_allclose(getattr(g.policy, k)[u].detach().cpu().numpy(), p.detach().numpy(),
                                           rtol=1e-3, atol=1e-5)
