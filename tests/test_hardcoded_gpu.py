"""HardcodedFixPriceEnvironment (SchedulingEnvironment.py:439-456) with the hard-coded agents acting inside
the env kernel (ms_actions acceptor = offer_core = NULL): closed-loop trajectories, no host actions,
bit-exact against the object-faithful restatement's HardcodedOfferer / HardcodedAcceptor
(oracle/pyref.py, HardcodedModules.py:16-109) on the same env streams."""
import numpy as np
import pytest

from oracle import pyref
from tests.test_env_gpu import _compare_state

pytestmark = pytest.mark.gpu

CASES = {
    "cfg1": None,
    "cfg2": None,
    "cfg3_fixed": dict(n_agents=8, n_cores=8, collection_length=3, priorities=[2, 4, 6, 8, 10, 12], lengths=[5] * 6,
                       fix_prices=[1, 3, 5, 7, 9, 11], probabilities=[0.25, 0.25, 0.125, 0.125, 0.125, 0.125]),
    "ties": dict(n_agents=3, n_cores=4, collection_length=3, priorities=[4, 8], lengths=[4, 8], fix_prices=[2, 4],
                 probabilities=[0.5, 0.5], new_jobs=2),
}


def _pcfg(abi, cfg, kw):
    K = cfg.n_kinds
    probs = list(kw["probabilities"]) if kw else list(abi.README_JOBS["probabilities"])
    return pyref.Config(cfg.n_agents, cfg.n_cores, cfg.collection_length, list(cfg.job_priority[:K]),
                        list(cfg.job_length[:K]), probs, fix_prices=list(cfg.fix_price[: cfg.n_fix_prices]),
                        new_jobs=cfg.new_jobs_per_round, reward_multiplier=cfg.reward_multiplier,
                        episode_length=cfg.episode_length)


@pytest.mark.parametrize("name", list(CASES))
def test_hardcoded_agents_closed_loop(ms, name):
    abi = ms.abi
    kw = CASES[name]
    cfg = abi.named_config(name) if kw is None else abi.make_config(**kw)
    s = abi.config_shape(cfg)
    E, T, seed = 8, 300, 21
    genv = ms.BatchedEnv(cfg, E, seed=seed)
    worlds = [pyref.PyWorld(_pcfg(abi, cfg, kw), seed + e) for e in range(E)]
    obs = genv.obs_buffers(auctioneer=True)
    genv.reset(obs)
    accepted = 0
    for t in range(T):
        gobs, grew, gev = genv.step(None, None, obs=obs, events=genv.event_buffers())
        ga = gobs["acceptor"].cpu().numpy()
        go = gobs["offer"].cpu().numpy()
        for e in range(E):
            acc, off = worlds[e].hardcoded_agent_actions()
            (r_acc, r_off, _), rew, _, _ = worlds[e].step(acc, off)
            accepted += len(worlds[e].accepted)
            assert np.array_equal(ga[e, :, :, : s["acc_obs_dim"]], np.array(r_acc)), (t, e)
            assert np.array_equal(go[e, :, :, : s["off_obs_dim"]], np.array(r_off)), (t, e)
            np.testing.assert_array_equal(grew["acceptor"][e].cpu().numpy(), rew[1][..., 0])
        if t % 60 == 0 or t == T - 1:
            _compare_state(genv.export_state(), [_pyref_export(w) for w in worlds], E)
    assert genv.flags() == 0 and accepted > 0


def _pyref_export(w):
    """pyref state in the oracle export layout (the keys _compare_state reads)."""
    st = w.state()
    C, N, L = w.C, w.N, w.L
    out = {k: np.asarray(st[k]) for k in ("core_owner", "core_kind", "core_rem", "core_birth", "slot_kind", "slot_rem",
                                          "slot_wait", "slot_birth", "offer_core", "offer_recip", "offer_price")}
    out["round"] = st["round"]
    cap = 128
    liab = np.zeros((C, cap, 5), np.int32)
    out["liab_n"] = np.array([len(x) for x in st["liab"]])
    for c in range(C):
        for i, entry in enumerate(st["liab"][c]):
            liab[c, i] = entry
    out["liab"] = liab
    words = st["mt_state"][1]
    out["mt"] = np.array(words[:624], dtype=np.uint32)
    out["mt_index"] = words[624]
    return out


def test_hardcoded_agents_full_size_cfg2_sampled(ms):
    """cfg2's 4096 replicas driven by the in-kernel hard-coded agents for 120 rounds: sampled replicas
    bit-exact against the restatement, and a second run from the same seed identical."""
    abi = ms.abi
    cfg = abi.named_config("cfg2")
    E, T, seed = 4096, 120, 5
    sample = [0, 1, 2047, 4095]
    runs = []
    for _ in range(2):
        genv = ms.BatchedEnv(cfg, E, seed=seed)
        obs = genv.obs_buffers()
        genv.reset(obs)
        for t in range(T):
            genv.step(None, None, obs=obs)
        runs.append((genv.export_state(), obs["acceptor"].cpu().numpy()))
        assert genv.flags() == 0
    worlds = [pyref.PyWorld(_pcfg(abi, cfg, None), seed + e) for e in sample]
    for t in range(T):
        for w in worlds:
            acc, off = w.hardcoded_agent_actions()
            w.step(acc, off)
    st = {k: v[sample] for k, v in runs[0][0].items()}
    _compare_state(st, [_pyref_export(w) for w in worlds], len(sample))
    for k in runs[0][0]:
        assert np.array_equal(runs[0][0][k], runs[1][0][k]), k
    assert np.array_equal(runs[0][1], runs[1][1])
