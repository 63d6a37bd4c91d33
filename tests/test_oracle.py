"""The oracle itself: RNG pinned to CPython's stdlib vectors, C restatement
cross-checked against the object-faithful Python restatement (oracle/pyref.py)."""
import json
import os
import random

import numpy as np
import pytest

from oracle import pyref
from tests.drivers import offer_counts_from_obs, random_actions

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _mt_cases():
    with open(os.path.join(GOLDEN, "mt_vectors.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", _mt_cases(), ids=lambda c: "seed%d" % c["seed"])
def test_mt_matches_cpython_vectors(oracle, case):
    cfg = oracle.abi.named_config("cfg1")
    st, idx = oracle.mt_seed_state(case["seed"])
    assert list(st[:8]) == case["state_words_head"]
    assert idx == case["state_index"]
    env = oracle.OracleEnv(cfg, case["seed"])
    assert [env.genrand() for _ in range(len(case["genrand"]))] == case["genrand"]
    env = oracle.OracleEnv(cfg, case["seed"])
    assert [env.random().hex() for _ in range(len(case["random"]))] == case["random"]
    env = oracle.OracleEnv(cfg, case["seed"])
    assert [env.randbelow(n) for n in case["randbelow_n"]] == case["randbelow"]
    # random.sample(pop, 1) and randint(a, b) are one _randbelow each
    env = oracle.OracleEnv(cfg, case["seed"])
    assert [env.randbelow(n) for n in case["sample1_n"]] == case["sample1"]
    env = oracle.OracleEnv(cfg, case["seed"])
    assert [a + env.randbelow(b - a + 1) for a, b in case["randint_ab"]] == case["randint"]


def test_mt_matches_live_cpython(oracle):
    """Same check against this interpreter's random module for extra seeds."""
    cfg = oracle.abi.named_config("cfg1")
    for seed in (3, 7, 99, 2**33 + 1):
        r = random.Random(seed)
        env = oracle.OracleEnv(cfg, seed)
        for _ in range(1300):
            assert env.genrand() == r.getrandbits(32)


def _pyref_config(cfg, abi):
    s = abi.config_shape(cfg)
    K = cfg.n_kinds
    probs = []
    prev = 0.0
    for i in range(K):  # recover per-kind probabilities for pyref (it re-accumulates)
        probs.append(cfg.acc_probability[i] - prev)
        prev = cfg.acc_probability[i]
    return s, pyref.Config(
        n_agents=cfg.n_agents, n_cores=cfg.n_cores, collection_length=cfg.collection_length,
        priorities=list(cfg.job_priority[:K]), lengths=list(cfg.job_length[:K]), probabilities=probs,
        fix_prices=list(cfg.fix_price[: cfg.n_fix_prices]), free_prices=bool(cfg.free_prices),
        commercial=bool(cfg.commercial_reward), net_zero_offer_reward=cfg.net_zero_offer_reward,
        new_jobs=cfg.new_jobs_per_round, reward_multiplier=cfg.reward_multiplier,
        episode_length=cfg.episode_length)


CROSS_CONFIGS = [
    ("cfg1", {}),
    ("cfg2", {}),
    ("small_free_commercial", dict(n_agents=3, n_cores=2, collection_length=2, priorities=[2, 4, 8],
                                   lengths=[5, 5, 5], probabilities=[0.5, 0.25, 0.25], free_prices=True,
                                   commercial=True)),
    ("small_free_noncommercial", dict(n_agents=2, n_cores=3, collection_length=3, priorities=[5],
                                      lengths=[5], probabilities=[1.0], free_prices=True, commercial=False)),
    ("two_jobs_per_round", dict(n_agents=3, n_cores=3, collection_length=4, priorities=[3, 10],
                                lengths=[6, 3], fix_prices=[2, 7], probabilities=[0.8, 0.2], new_jobs=2,
                                reward_multiplier=2)),
]


@pytest.mark.parametrize("name,kw", CROSS_CONFIGS, ids=[c[0] for c in CROSS_CONFIGS])
def test_c_oracle_matches_object_faithful_restatement(oracle, name, kw):
    abi = oracle.abi
    cfg = abi.named_config(name) if not kw else abi.make_config(**kw)
    # probabilities must be exactly recoverable for pyref: rebuild from kw when given
    s, pcfg = _pyref_config(cfg, abi)
    if kw:
        pcfg.probabilities = list(kw["probabilities"])
    elif name in ("cfg1", "cfg2"):
        pcfg.probabilities = list(abi.README_JOBS["probabilities"])
    N, C, L, O = s["N"], s["C"], s["L"], s["O"]
    for seed in (0, 1, 5):
        cenv = oracle.OracleEnv(cfg, seed)
        penv = pyref.PyWorld(pcfg, seed)
        rng = np.random.default_rng(1000 + seed)
        obs = cenv.observe()
        for t in range(400):
            acc, off, price = random_actions(rng, offer_counts_from_obs(obs["acceptor"], O), N, C, L, O,
                                             bool(cfg.free_prices), s["price_actions"] - 1)
            cres = cenv.step(acc, off, price)
            if cfg.free_prices:
                poff = [[(int(off[a, l]), int(price[a, l])) for l in range(L)] for a in range(N)]
            else:
                poff = off.tolist()
            (pacc, poffo, pauct), prew, pq, _ = penv.step(acc.tolist(), poff)
            obs = cenv.observe()
            assert obs["acceptor"].tolist() == pacc, (name, seed, t)
            assert obs["offer"].tolist() == poffo, (name, seed, t)
            assert obs["auctioneer"].tolist() == pauct, (name, seed, t)
            off_r, acc_r, auct_r, agent_r, term_rev = prew
            if cfg.free_prices:
                np.testing.assert_array_equal(cres["offer"], off_r[0][..., 0])
                np.testing.assert_array_equal(cres["price"], off_r[1][..., 0])
            else:
                np.testing.assert_array_equal(cres["offer"], off_r[..., 0])
                assert cres["termination_revenue"] == term_rev
            np.testing.assert_array_equal(cres["acceptor"], acc_r[..., 0])
            np.testing.assert_array_equal(cres["auctioneer"], auct_r)
            np.testing.assert_array_equal(cres["agent"], agent_r)
            assert list(cres["quality"]) == pq
            cs = cenv.export_state()
            ps = penv.state()
            for k in ("core_owner", "core_kind", "core_rem", "slot_kind", "slot_rem", "slot_wait",
                      "offer_core", "offer_recip", "offer_price"):
                assert np.asarray(cs[k]).tolist() == ps[k], (k, t)
            assert int(cs["round"]) == ps["round"]
            for c in range(C):
                n = int(cs["liab_n"][c])
                assert [tuple(x) for x in cs["liab"][c, :n].tolist()] == ps["liab"][c]
            words = ps["mt_state"][1]
            assert list(cs["mt"]) == list(words[:624]) and int(cs["mt_index"]) == words[624]
        assert cenv.flags == 0


def test_settlement_rounds_the_double_product(oracle):
    """KAT: round(7/6 * 105) = 123 with the float64 product (exact rational gives 122.5 -> 122)."""
    assert round(7 / 6 * 105) == 123
    abi = oracle.abi
    cfg = abi.make_config(2, 1, 1, priorities=[12], lengths=[6], probabilities=[1.0], free_prices=True)
    env = oracle.OracleEnv(cfg, 0)
    st = env.export_state()
    # core 0 owned by agent 1 running a job with 1 round left; one liability entry
    # (offerer 1 -> auctioneer, price 7, necT 6) accepted at round 0; now round 104.
    st["round"] = 104
    st["core_owner"][0] = 1
    st["core_kind"][0] = 0
    st["core_rem"][0] = 1
    st["core_birth"][0] = 0
    st["liab_n"][0] = 1
    st["liab"][0, 0] = [1, 0, 7, 6, 0]
    env.import_state(st)
    res = env.step(np.array([[1], [1]]), np.array([[1], [1]]), np.array([[-5], [-5]]), auct=np.array([1]))
    # T = (104 + 1) - 0 = 105 ; traded = round(7/6*105) = 123
    assert res["acceptor"][0, 0] == 12 - 123
    assert res["agent"][0] == -123  # free prices: no termination reward in agentReward (Reward.py:59-63)
    assert res["auctioneer"][0] == 123
