"""Episode metrics (§8(f) row 3): the env kernel's per-replica accumulators (ms_env_metrics) turned
into trainPPO.py's per-episode values (marl-scheduling_amd/metrics.py) against the driver's own
code restated on the object-faithful world (oracle/metrics_ref.py), same seeds and actions."""
import importlib
import os

import numpy as np
import pytest
import torch

from oracle import pyref
from oracle.metrics_ref import EpisodeRecorder
from tests.drivers import offer_counts_from_obs, random_actions

pytestmark = pytest.mark.gpu

CASES = {
    "fixed": dict(n_agents=3, n_cores=3, collection_length=3, priorities=[3, 10, 6], lengths=[6, 3, 4],
                  fix_prices=[2, 7, 4], probabilities=[0.5, 0.25, 0.25], episode_length=25),
    "free_commercial": dict(n_agents=4, n_cores=3, collection_length=2, priorities=[2, 4, 8, 8],
                            lengths=[5, 5, 3, 3], probabilities=[0.25, 0.25, 0.25, 0.25], free_prices=True,
                            commercial=True, episode_length=20),
}


def _close(a, b, rel=1e-6):
    if a is None or b is None:
        assert a is None and b is None, (a, b)
        return
    assert abs(float(a) - float(b)) <= rel * max(1.0, abs(float(b))), (a, b)


@pytest.mark.parametrize("name", list(CASES))
def test_episode_metrics_match_driver(ms, name):
    abi = ms.abi
    mx = importlib.import_module("marl-scheduling_amd.metrics")
    kw = dict(CASES[name])
    cfg = abi.make_config(**kw)
    s = abi.config_shape(cfg)
    N, C, L, O = s["N"], s["C"], s["L"], s["O"]
    T = kw["episode_length"]
    E, seed, episodes, slots = 5, 11, 3, 2
    pcfg = pyref.Config(n_agents=N, n_cores=C, collection_length=L, priorities=kw["priorities"],
                        lengths=kw["lengths"], probabilities=kw["probabilities"],
                        fix_prices=kw.get("fix_prices", []), free_prices=kw.get("free_prices", False),
                        commercial=kw.get("commercial", True), episode_length=T)
    genv = ms.BatchedEnv(cfg, E, seed=seed)
    worlds = [pyref.PyWorld(pcfg, seed + e) for e in range(E)]
    dev = genv.device
    mbuf = genv.metrics_buffer(slots)
    free = bool(cfg.free_prices)
    rng = np.random.default_rng(5)
    obs = [w.observe() for w in worlds]
    for ep in range(episodes):
        recs = [EpisodeRecorder(w, free) for w in worlds]
        for t in range(T):
            acts = [random_actions(rng, offer_counts_from_obs(np.array(obs[e][0]), O), N, C, L, O, free,
                                   s["price_actions"] - 1, accept_bias=0.7) for e in range(E)]
            acc = torch.tensor(np.stack([a[0] for a in acts]), dtype=torch.int8, device=dev)
            off = torch.tensor(np.stack([a[1] for a in acts]), dtype=torch.int8, device=dev)
            pr = torch.tensor(np.stack([a[2] for a in acts]), dtype=torch.int8, device=dev) if free else None
            genv.step(acc, off, pr, events=dict(metrics=mbuf))
            for e in range(E):
                a, o, p = acts[e]
                poff = [[(int(o[i, l]), int(p[i, l])) for l in range(L)] for i in range(N)] if free else o.tolist()
                out = worlds[e].step(a.tolist(), poff)
                recs[e].add(out)
                obs[e] = out[0]
        slot = ep % slots
        got = mx.episode_values(mx.view(mbuf[slot].cpu().numpy()), cfg, T, N, C, L)
        mbuf[slot].zero_()
        for e in range(E):
            want = recs[e].finish(pcfg, T)
            g = got[e]
            assert g["rounds"] == T
            for k in ("acceptorRew", "coreChooserRew", "priceChooserRew", "auctioneerRew", "acceptionQuality",
                      "acceptionAmount", "terminationRevenues", "tradeRevenues"):
                _close(g[k], want[k])
            for k in ("prices", "dwellTimes"):
                assert len(g[k]) == len(want[k])
                for x, y in zip(g[k], want[k]):
                    _close(x, y, 1e-12)
            np.testing.assert_allclose(g["agentRew"], want["agentRew"], rtol=1e-12)
        # the next episode's slot starts from zero (the kernel adds into slot (round / T) % slots)
    assert genv.flags() == 0
    d = mx.args_dict([got], cfg, params=dict(episodeLength=T))
    assert set(d) >= {"acceptorRew", "prices", "dwellTimes", "meanJob", "params", "acceptionQuality"}


def test_trainer_collects_args_dict(ms):
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    t = tr_mod.Trainer.from_named("cfg3", n_envs=64, update_step=20, seed=2, device="cuda:0", metrics=True,
                                  episode_length=10)
    t.iteration()
    t.iteration()
    d = t.args_dict()
    assert len(d["acceptorRew"]) == 4 and len(d["prices"][0]) == 6
    assert all(isinstance(v, float) for v in d["acceptionAmount"])


def test_trainer_pickles_args_dict_like_trainppo(ms, tmp_path):
    """save_args_dict writes the first free data{i}.pkl (trainPPO.py:245-251) with the argsDict keys
    Plot.py reads."""
    import pickle
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    t = tr_mod.Trainer.from_named("cfg3", n_envs=32, update_step=20, seed=2, device="cuda:0", metrics=True,
                                  episode_length=10)
    t.iteration()
    (tmp_path / "data0.pkl").write_bytes(b"taken")
    p = t.save_args_dict(str(tmp_path))
    assert os.path.basename(p) == "data1.pkl"
    with open(p, "rb") as f:  # our own file, written just above
        d = pickle.load(f)
    assert set(d) >= {"plotPath", "acceptorRew", "coreChooserRew", "priceChooserRew", "prices", "auctioneerRew",
                      "dwellTimes", "meanJob", "agentRew", "acceptionQuality", "acceptionAmount",
                      "terminationRevenues", "tradeRevenues", "params"}
    assert len(d["acceptorRew"]) == 2 and d["params"]["episodeLength"] == 10
