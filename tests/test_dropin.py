"""The E = 1 drop-in modules (marl-scheduling_amd/dropin: world, SchedulingEnvironment, PPOmodules)
driven the way trainPPO.py:133-227 drives the reference, against the object-faithful restatement
(oracle/pyref.py) and the torch PPO restatement (oracle/ppo_ref.py)."""
import os
import random
import statistics
import sys

import numpy as np
import pytest
import torch

from tests.drivers import random_actions

DROPIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-scheduling_amd", "dropin")


def _mods():
    if DROPIN not in sys.path:
        sys.path.insert(0, DROPIN)
    import PPOmodules
    import SchedulingEnvironment
    import world

    return world, SchedulingEnvironment, PPOmodules


def world_params(N=3, C=3, L=2, free=False, prios=(3, 10), lens=(6, 3), probs=(0.8, 0.2), fix=(2, 7), ep=100):
    return {"num_episodes": 1, "episodeLength": ep, "numberOfAgents": N, "numberOfCores": C,
            "possibleJobPriorities": list(prios), "possibleJobLengths": list(lens), "collectionLength": L,
            "probabilities": list(probs), "newJobsPerRoundPerAgent": 1, "rewardMultiplier": 1, "freePrices": free,
            "fixPricesList": list(fix), "maxVisibleOffers": 4}


def rl_params(acc_k=3, off_k=3, raw_k=3, cs=2, acc_gamma=0.9):
    return {"LR_ACTOR": 0.003, "LR_CRITIC": 0.01, "EPS_CLIP": 0.2, "ACCEPTOR_GAMMA": acc_gamma,
            "netZeroOfferReward": 0.5, "OFFER_GAMMA": 0.5, "RAW_K_EPOCHS": raw_k, "RANDOMPOLICY": False,
            "UPDATE_STEP": 200, "globallySharedParameters": False, "locallySharedParameters": False,
            "ACCEPTOR_K_EPOCHS": acc_k, "OFFER_K_EPOCHS": off_k, "CENTRALISATION_SAMPLE": cs}


def test_dropin_modules_keep_the_reference_names():
    world, env_mod, ppo_mod = _mods()
    for name in ("SchedulingEnv", "PPOSchedulingEnv", "PPODividedFixedPriceEnv", "PPODividedFreePriceEnv",
                 "GloballySharedParamsDividedFixedPriceEnv", "LocallySharedParamsDividedFixedPriceEnv"):
        assert hasattr(env_mod, name), name
    for name in ("ExperienceBuffer", "ActorCritic"):
        assert hasattr(ppo_mod, name)
    w = world.World(world_params())
    assert w.round == 0 and w.maxAmountOfOffersToOneAgent == 6 and w.accProbabilities == [0.8, 1.0]
    assert w.acceptedOffers == [] and w.verweilzeiten == []
    if not torch.cuda.is_available():  # no CPU fallback
        with pytest.raises(RuntimeError):
            env_mod.PPODividedFixedPriceEnv(w, rl_params())


def _pyref_config(wp, free, commercial=True):
    from oracle.pyref import Config

    return Config(wp["numberOfAgents"], wp["numberOfCores"], wp["collectionLength"], wp["possibleJobPriorities"],
                  wp["possibleJobLengths"], wp["probabilities"], fix_prices=wp["fixPricesList"], free_prices=free,
                  commercial=commercial, net_zero_offer_reward=0.5, episode_length=wp["episodeLength"])


def _as_lists(nested):
    return [[t.tolist() for t in agent] for agent in nested]


ENV_CASES = [
    ("fixed", dict(N=3, C=3, L=2)),
    ("fixed", dict(N=4, C=2, L=3, prios=(3, 10, 5), lens=(6, 3, 2), probs=(0.5, 0.3, 0.2), fix=(2, 7, 3), ep=37)),
    ("free", dict(N=3, C=4, L=2)),
    ("free_noncommercial", dict(N=2, C=2, L=2, prios=(2, 4, 6, 8, 10, 12), lens=(5,) * 6, probs=(1 / 6,) * 6,
                                fix=(1,) * 6)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("mode,kw", ENV_CASES)
def test_dropin_env_matches_object_restatement(mode, kw):
    from oracle.pyref import PyWorld

    world, env_mod, _ = _mods()
    free = mode != "fixed"
    commercial = mode != "free_noncommercial"
    wp = world_params(free=free, **kw)
    seed = 4321
    random.seed(seed)
    torch.manual_seed(0)
    w = world.World(wp)
    env = env_mod.PPODividedFreePriceEnv(w, rl_params(), commercial) if free else \
        env_mod.PPODividedFixedPriceEnv(w, rl_params())
    pw = PyWorld(_pyref_config(wp, free, commercial), seed)
    N, C, L = wp["numberOfAgents"], wp["numberOfCores"], wp["collectionLength"]
    O = N * L
    rng = np.random.default_rng(7)
    acc_obs, off_obs, auct_obs = env.reset()
    ref = pw.observe()
    assert _as_lists(acc_obs) == ref[0] and _as_lists(off_obs) == ref[1]
    env.terminationRevenues = 0
    term_rev = 0
    for t in range(160):
        counts = [[sum(1 for v in row.tolist()[4::2] if v != -2) for row in agent] for agent in acc_obs]
        acc, off, price = random_actions(rng, counts, N, C, L, O, free, max(wp["possibleJobPriorities"]))
        acc_l = acc.tolist()
        off_l = [[(int(off[a, j]), int(price[a, j])) for j in range(L)] for a in range(N)] if free else off.tolist()
        auct = w.auctioneer.getAuctioneerAction(auct_obs)
        assert auct == pw.auctioneer_actions()
        out = env.step(off_l, acc_l, auct)
        (r_obs, r_rew, r_q, r_done) = pw.step(acc_l, off_l if not free else [[list(p) for p in row] for row in off_l],
                                              auct)
        acc_obs, off_obs, auct_obs = out[0], out[1], out[2]
        assert all(x.dtype == torch.int64 for agent in acc_obs for x in agent)
        assert _as_lists(acc_obs) == r_obs[0], t
        assert _as_lists(off_obs) == r_obs[1], t
        assert [x.tolist() for x in auct_obs] == r_obs[2], t
        off_r, acc_r, auct_r, agent_r, rev = r_rew
        term_rev += rev
        if free:
            assert out[3][0].dtype == np.float64 and out[3][0].shape == (N, L, 1)
            np.testing.assert_array_equal(out[3][0], off_r[0])
            np.testing.assert_array_equal(out[3][1], off_r[1])
        else:
            assert out[3].dtype == np.int64 and out[3].shape == (N, L, 1)
            np.testing.assert_array_equal(out[3], off_r)
        assert out[4].dtype == np.int64 and out[4].shape == (N, C, 1)
        np.testing.assert_array_equal(out[4], acc_r)
        np.testing.assert_array_equal(out[5], auct_r)
        np.testing.assert_array_equal(out[6], agent_r)
        assert out[7] == ((statistics.mean(r_q) if r_q else None), len(r_q))
        assert out[8] == r_done and w.round == pw.round
        assert random.getstate() == pw.rng.getstate(), t  # the global stream IS the env stream
        got = [(o.offererID, o.recipientID, o.coreID, o.queuePosition, o.offeredReward, o.prio1, o.jobKind)
               for o in w.acceptedOffers]
        want = [(o.offerer, o.recipient, o.core_id, o.queue_pos, o.price, o.prio1, o.kind) for o in pw.accepted]
        assert got == want, t
        env.saveRewards(out[3], out[4], out[6])
    assert [tuple(v) for v in w.verweilzeiten] == pw.dwell
    if not free:
        assert env.terminationRevenues == term_rev


def _snapshot(units, kind):
    u = units[kind]
    T = u.T
    return (u.states[:T].cpu().clone(), u.actions[:T].cpu().long().clone(), u.logprobs[:T].cpu().clone(),
            np.stack(u.rewards).copy())


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["divided", "global", "local"])
def test_dropin_ppo_update_matches_reference(arch):
    from oracle.ppo_ref import RefPPO

    world, env_mod, ppo_mod = _mods()
    N, C, L = 3, 2, 2
    wp = world_params(N=N, C=C, L=L)
    rp = rl_params(acc_k=2, off_k=2, cs=2)
    cls = {"divided": env_mod.PPODividedFixedPriceEnv, "global": env_mod.GloballySharedParamsDividedFixedPriceEnv,
           "local": env_mod.LocallySharedParamsDividedFixedPriceEnv}[arch]
    random.seed(11)
    torch.manual_seed(5)
    w = world.World(wp)
    env = cls(w, rp)
    s = env._eng.env.shape
    dims = dict(acc=(s.acc_obs_dim, s.acc_actions), off=(s.off_obs_dim, s.off_actions))
    # reference construction order on the same torch seed
    torch.manual_seed(5)
    G = dict(divided=dict(acc=N * C, off=N * L), local=dict(acc=N, off=N), **{"global": dict(acc=1, off=1)})[arch]
    order = {"divided": [k for _ in range(N) for k in ["acc"] * C + ["off"] * L],
             "local": [k for _ in range(N) for k in ["acc", "off"]], "global": ["acc", "off"]}[arch]
    refs = dict(acc=[], off=[])
    for k in order:
        gam = rp["ACCEPTOR_GAMMA"] if k == "acc" else rp["OFFER_GAMMA"]
        K = rp["ACCEPTOR_K_EPOCHS"] if k == "acc" else rp["OFFER_K_EPOCHS"]
        refs[k].append(RefPPO(dims[k][0], dims[k][1], 0.003, 0.01, gam, 0.2, K))
    for k in ("acc", "off"):
        assert len(refs[k]) == G[k]
        for g, r in enumerate(refs[k]):
            for name, v in r.policy.flat().items():
                torch.testing.assert_close(getattr(env._units[k].group.policy, name)[g].cpu(), v.detach(), rtol=0,
                                           atol=0)
    acc_obs, off_obs, auct_obs = env.reset()
    T = 30
    for _ in range(T):
        acc_l, off_l = env.getActionForAllAgents(acc_obs, off_obs)
        auct = w.auctioneer.getAuctioneerAction(auct_obs)
        out = env.step(off_l, acc_l, auct)
        acc_obs, off_obs, auct_obs = out[0], out[1], out[2]
        env.saveRewards(out[3], out[4], out[6])
    snap = {k: _snapshot(env._units, k) for k in ("acc", "off")}
    # the sub-unit draws the update will make, from a copy of the global stream
    st = random.getstate()
    CS = rp["CENTRALISATION_SAMPLE"]
    if arch == "divided":
        sel = dict(acc=[list(range(N * C))], off=[list(range(N * L))])
    elif arch == "local":
        ad, od = [], []
        for _ in range(N):
            ad.append([random.randint(0, C - 1) for _ in range(CS)])
            od.append([random.randint(0, L - 1) for _ in range(CS)])
        sel = dict(acc=[[a * C + ad[a][i] for a in range(N)] for i in range(CS)],
                   off=[[a * L + od[a][i] for a in range(N)] for i in range(CS)])
    else:
        sa, so = [], []
        for _ in range(CS):
            a = random.randint(0, N - 1)
            sa.append([a * C + random.randint(0, C - 1)])
        for _ in range(CS):
            a = random.randint(0, N - 1)
            so.append([a * L + random.randint(0, L - 1)])
        sel = dict(acc=sa, off=so)
    random.setstate(st)
    env.updateAgents()
    assert random.getstate() != st or arch == "divided"
    for k in ("acc", "off"):
        states, actions, lps, rews = snap[k]
        D = dims[k][0]
        for pick in sel[k]:
            for g, u in enumerate(pick):
                ref = refs[k][g]
                x = states[:, u, :D].float()
                ret = ref.returns(rews[:, u].tolist())
                ref.update(x, actions[:, u], lps[:, u], ret)
        for g, ref in enumerate(refs[k]):
            for name, v in ref.policy.flat().items():
                np.testing.assert_allclose(getattr(env._units[k].group.policy, name)[g].detach().cpu().numpy(),
                                           v.detach().numpy(), rtol=1e-4, atol=1e-5, err_msg="%s %s %d" % (k, name, g))
        assert env._units[k].T == 0 and env._units[k].rewards == []


@pytest.mark.gpu
@pytest.mark.parametrize("env_name", ["PPODividedFixedPriceEnv", "PPODividedFreePriceEnv",
                                      "GloballySharedParamsDividedFixedPriceEnv",
                                      "LocallySharedParamsDividedFixedPriceEnv",
                                      "LocallySharedParamsDividedFreePriceEnv", "PPOAggregatedFixPriceEnv",
                                      "PPOFullyAggregatedFixPriceEnv"])
def test_dropin_runs_the_trainppo_loop(env_name):
    """The loop body of trainPPO.py:133-216, unchanged, for 3 episodes with updates."""
    world, env_mod, _ = _mods()
    free = "Free" in env_name
    wp = world_params(N=2, C=2, L=2, free=free, ep=10)
    rp = rl_params(acc_k=1, off_k=1, raw_k=1)
    random.seed(0)
    torch.manual_seed(0)
    w = world.World(wp)
    env = getattr(env_mod, env_name)(w, rp, True) if free else getattr(env_mod, env_name)(w, rp)
    UPDATE_STEP = 2 * wp["episodeLength"]
    updates = 0
    for _ in range(3):
        newAcc, newOff, newAuct = env.reset()
        env.tradeRevenues = 0
        env.terminationRevenues = 0
        prices = []
        for _ in range(1000):
            acceptorActions, offerActions = env.getActionForAllAgents(newAcc, newOff)
            auctioneer_action = w.auctioneer.getAuctioneerAction(newAuct)
            (newAcc, newOff, newAuct, offerRewards, acceptorRewards, auctioneerReward, agentReward, acceptionQuality,
             done) = env.step(offerActions, acceptorActions, auctioneer_action)
            env.saveRewards(offerRewards, acceptorRewards, agentReward)
            if (w.round > 0) & (((w.round) % UPDATE_STEP) == 0):
                env.updateAgents()
                updates += 1
            for offer in w.acceptedOffers:
                prices.append((offer.offeredReward, offer.jobKind))
            sum(auctioneerReward.tolist())
            if done:
                break
    assert updates == 1 and w.round == 30
    for u in env._units.values():
        assert u.T == 10 and all(torch.isfinite(p).all() for p in u.group.policy.parameters())


@pytest.mark.gpu
@pytest.mark.parametrize("fully", [False, True])
def test_dropin_aggregated_env_matches_object_restatement(fully):
    """PPOAggregatedFixPriceEnv / PPOFullyAggregatedFixPriceEnv: observation containers (float32
    acceptor rows, int64 offer rows per agent) and getAggregatedFixedPricesReward arrays against the
    restatement, with the global random stream shared, and the nets in the reference's init order."""
    from oracle.pyref import PyWorld

    world, env_mod, _ = _mods()
    wp = world_params(N=2, C=2, L=2)
    seed = 99
    random.seed(seed)
    torch.manual_seed(3)
    w = world.World(wp)
    cls = env_mod.PPOFullyAggregatedFixPriceEnv if fully else env_mod.PPOAggregatedFixPriceEnv
    env = cls(w, rl_params())
    torch.manual_seed(3)
    ppo = __import__("marlsched_dropin").ppo
    O, N, C = 4, 2, 2
    da, do = C * (3 + 2 * O), 2 * C + 2 * 2
    first = ppo.reference_actor_critic_params(do + da, 25 * 9, 64) if fully else \
        ppo.reference_actor_critic_params(da, 25, 32)
    unit = env._units["fully" if fully else "acc"]
    for name, v in first.items():
        torch.testing.assert_close(getattr(unit.group.policy, name)[0].cpu(), v.detach(), rtol=0, atol=0)
    pw = PyWorld(_pyref_config(wp, False), seed)
    acc_obs, off_obs, auct_obs = env.reset()
    for t in range(120):
        pa, po, _ = pw.aggregated_obs()
        assert all(x.dtype == torch.float32 for x in acc_obs) and all(x.dtype == torch.int64 for x in off_obs)
        assert [x.tolist() for x in acc_obs] == pa and [x.tolist() for x in off_obs] == po, t
        acc_l, off_l = env.getActionForAllAgents(acc_obs, off_obs)
        auct = w.auctioneer.getAuctioneerAction(auct_obs)
        assert auct == pw.auctioneer_actions()
        out = env.step(off_l, acc_l, auct)
        _, (_, _, auct_r, agent_r, _), _, _ = pw.step(acc_l, off_l, auct)
        w_off, w_acc = pw.last_aggregated
        assert out[3].dtype == np.int64 and out[3].shape == (N, 1) and out[4].shape == (N, 1)
        np.testing.assert_array_equal(out[3], w_off)
        np.testing.assert_array_equal(out[4], w_acc)
        np.testing.assert_array_equal(out[5], auct_r)
        np.testing.assert_array_equal(out[6], agent_r)
        assert random.getstate() == pw.rng.getstate(), t
        env.saveRewards(out[3], out[4], out[6])
        acc_obs, off_obs, auct_obs = out[0], out[1], out[2]
    env.updateAgents()
    for u in env._units.values():
        assert u.T == 0 and all(torch.isfinite(p).all() for p in u.group.policy.parameters())


@pytest.mark.gpu
def test_dropin_hardcoded_env_matches_restatement():
    """trainPPO.py's loop with hardcodedAgents (SchedulingEnvironment.py:439-456) against the restatement's
    hard-coded agents on the same global stream."""
    from oracle.pyref import PyWorld

    world, env_mod, _ = _mods()
    wp = world_params(N=3, C=4, L=2, ep=25)
    seed = 77
    random.seed(seed)
    w = world.World(wp)
    env = env_mod.HardcodedFixPriceEnvironment(w, rl_params())
    pw = PyWorld(_pyref_config(wp, False), seed)
    acc_obs, off_obs, auct_obs = env.reset()
    for t in range(100):
        acc, off = env.getActionForAllAgents(acc_obs, off_obs)
        r_acc, r_off = pw.hardcoded_agent_actions()
        assert (acc, off) == (r_acc, r_off), t
        auct = w.auctioneer.getAuctioneerAction(auct_obs)
        out = env.step(off, acc, auct)
        (r_obs, _, _, _) = pw.step(r_acc, r_off, pw.auctioneer_actions())
        acc_obs, off_obs, auct_obs = out[0], out[1], out[2]
        assert _as_lists(acc_obs) == r_obs[0], t
        assert random.getstate() == pw.rng.getstate(), t
        env.saveRewards(out[3], out[4], out[6])
        env.updateAgents()
