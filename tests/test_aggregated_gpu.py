"""Aggregated / fully-aggregated agents (Agent.py:73-140, 359-492; Reward.py:92-143) on the device.

Agent action numbers are decoded on the device (ms_decode_aggregated), the divided env step runs,
and the aggregated observations (ms_aggregate_obs) and rewards (ms_reward_out.aggregated_*) are
compared bit for bit with the object-faithful restatement (oracle/pyref.py), replica by replica.
"""
import numpy as np
import pytest
import torch

from oracle import pyref

pytestmark = pytest.mark.gpu

CASES = {
    # README job set (cfg1 shape: 2 agents, 2 cores, collectionLength 2)
    "cfg1": dict(n_agents=2, n_cores=2, collection_length=2, priorities=[3, 10], lengths=[6, 3], fix_prices=[2, 7],
                 probabilities=[0.8, 0.2]),
    "three": dict(n_agents=3, n_cores=2, collection_length=2, priorities=[2, 9, 5], lengths=[4, 2, 3],
                  fix_prices=[1, 6, 3], probabilities=[0.5, 0.25, 0.25], reward_multiplier=2),
}


def _pcfg(kw):
    return pyref.Config(n_agents=kw["n_agents"], n_cores=kw["n_cores"], collection_length=kw["collection_length"],
                        priorities=kw["priorities"], lengths=kw["lengths"], probabilities=kw["probabilities"],
                        fix_prices=kw["fix_prices"], reward_multiplier=kw.get("reward_multiplier", 1))


@pytest.mark.parametrize("fully", [False, True])
@pytest.mark.parametrize("name", list(CASES))
def test_aggregated_env_matches_restatement(ms, name, fully):
    kw = CASES[name]
    cfg = ms.abi.make_config(**kw)
    E, T, seed = 12, 150, 11
    env = ms.BatchedEnv(cfg, E, seed=seed)
    N, C, L, O = env.N, env.C, env.L, env.O
    n_acc, n_off = env.aggregated_action_counts()
    worlds = [pyref.PyWorld(_pcfg(kw), seed + e) for e in range(E)]
    obs = env.reset(env.obs_buffers())
    rew = env.reward_buffers(aggregated=True)
    dims = env.aggregated_dims()
    rng = np.random.default_rng(5)
    bad = torch.zeros(1, dtype=torch.int32, device=env.device)
    for t in range(T):
        agg = env.aggregate_obs(obs, kinds=("acceptor", "offer", "fully"))
        for e in range(E):
            pa, po, pf = worlds[e].aggregated_obs()
            for k, want in (("acceptor", pa), ("offer", po), ("fully", pf)):
                got = agg[k][e, :, : dims[k][0]].cpu().numpy()
                np.testing.assert_array_equal(got, np.array(want), err_msg="%s obs env %d round %d" % (k, e, t))
                assert not agg[k][e, :, dims[k][0]:].any()
        # a bias towards low acceptor numbers (digit 0 = accept the first offer) makes executions common
        if fully:
            nums = rng.integers(0, n_acc * n_off, (E, N))
            acc_n, off_n = nums // n_off, nums % n_off
            dev = torch.tensor(nums, dtype=torch.int32, device=env.device)
        else:
            acc_n = np.where(rng.random((E, N)) < 0.5, rng.integers(0, n_acc, (E, N)), rng.integers(0, 2, (E, N)))
            off_n = rng.integers(0, n_off, (E, N))
            dev = torch.tensor(np.stack([acc_n, off_n]), dtype=torch.int32, device=env.device)
        acc_a, off_a = env.decode_aggregated(dev.contiguous(), fully, n_bad=bad)
        acc_h, off_h = acc_a.cpu().numpy(), off_a.cpu().numpy()
        for e in range(E):
            for a in range(N):
                assert acc_h[e, a].tolist() == pyref.number_to_nd_action(int(acc_n[e, a]), O + 1, C)
                assert off_h[e, a].tolist() == pyref.number_to_nd_action(int(off_n[e, a]), C + 1, L)
        obs, rew, _ = env.step(acc_a, off_a, obs=obs, rewards=rew)
        agg_off = rew["aggregated_offer"].cpu().numpy()
        agg_acc = rew["aggregated_acceptor"].cpu().numpy()
        agent = rew["agent"].cpu().numpy()
        for e in range(E):
            _, (off_r, acc_r, auct_r, agent_r, _), _, _ = worlds[e].step(acc_h[e].tolist(), off_h[e].tolist())
            w_off, w_acc = worlds[e].last_aggregated
            np.testing.assert_array_equal(agg_off[e], w_off[:, 0], err_msg="offer reward env %d round %d" % (e, t))
            np.testing.assert_array_equal(agg_acc[e], w_acc[:, 0], err_msg="acceptor reward env %d round %d" % (e, t))
            np.testing.assert_array_equal(agent[e], agent_r)
    assert int(bad.item()) == 0
    assert env.flags() == 0


def test_decode_rejects_out_of_range_numbers(ms):
    kw = CASES["cfg1"]
    env = ms.BatchedEnv(ms.abi.make_config(**kw), 3, seed=0)
    n_acc, n_off = env.aggregated_action_counts()
    nums = torch.tensor([[0, n_acc * n_off], [-1, 5], [n_acc * n_off - 1, 7]], dtype=torch.int32,
                        device=env.device)
    bad = torch.zeros(1, dtype=torch.int32, device=env.device)
    acc, off = env.decode_aggregated(nums, True, n_bad=bad)
    assert int(bad.item()) == 2
    assert acc[0, 1].tolist() == [env.O] * env.C and off[1, 0].tolist() == [env.C] * env.L
    assert acc[2, 0].tolist() == [env.O] * env.C and off[2, 0].tolist() == [env.C] * env.L  # the maximum number


@pytest.mark.parametrize("fully", [False, True])
def test_aggregated_trainer_rollout_replays_on_the_restatement(ms, fully):
    """AggregatedTrainer: the recorded action numbers, replayed through numberToNDimensionalAction on
    the object-faithful restatement, reproduce the recorded observations and saved rewards
    (SchedulingEnvironment.py:223-247); then the PPO update runs and the second iteration continues."""
    import importlib
    agg = importlib.import_module("marl-scheduling_amd.aggregated")
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    kw = CASES["cfg1"]
    cfg = ms.abi.make_config(**kw)
    E, T = 6, 40
    tr = agg.AggregatedTrainer(cfg, E, fully=fully, hyper=tr_mod.Hyper(update_step=T), seed=2)
    env = tr.env
    N, C, L, O = env.N, env.C, env.L, env.O
    n_acc, n_off = env.aggregated_action_counts()
    base = tr_mod.env_seed(2, 0, E)
    worlds = [pyref.PyWorld(_pcfg(kw), base + e) for e in range(E)]
    for t in range(T):
        tr.round(t)
    dims = env.aggregated_dims()
    units = {k: (u.obs.cpu().numpy(), u.actions.cpu().numpy(), u.rewards.cpu().numpy()) for k, u in tr.units.items()}
    for t in range(T):
        for e in range(E):
            pa, po, pf = worlds[e].aggregated_obs()
            want = dict(acceptor=pa, offer=po, fully=pf)
            for k, (obs, _, _) in units.items():
                np.testing.assert_array_equal(obs[t, e, :, : dims[k][0]], np.array(want[k]), err_msg="%s t%d" % (k, t))
            if fully:
                nums = units["fully"][1][t, e]
                acc_n, off_n = nums // n_off, nums % n_off
            else:
                acc_n, off_n = units["acceptor"][1][t, e], units["offer"][1][t, e]
            acc = [pyref.number_to_nd_action(int(acc_n[a]), O + 1, C) for a in range(N)]
            off = [pyref.number_to_nd_action(int(off_n[a]), C + 1, L) for a in range(N)]
            _, (_, _, _, agent_r, _), _, _ = worlds[e].step(acc, off)
            w_off, _ = worlds[e].last_aggregated
            if fully:
                np.testing.assert_array_equal(units["fully"][2][t, e], agent_r + w_off[:, 0])
            else:
                np.testing.assert_array_equal(units["acceptor"][2][t, e], agent_r)
                np.testing.assert_array_equal(units["offer"][2][t, e], w_off[:, 0])
    losses = tr.update()
    for v in losses.values():
        assert torch.isfinite(v).all()
    tr.iteration()
    assert tr.bad_actions() == 0 and tr.flags() == 0 and env.round == 2 * T
