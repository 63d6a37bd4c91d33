"""Bit-exact parity of the HIP env step (ms_env_step) with the CPU restatement.

Same seeds, same actions: observations, rewards, events and the full state
(including every MT19937 word) must be identical after every round.
"""
import numpy as np
import pytest
import torch

from tests.drivers import offer_counts_from_obs, random_actions

pytestmark = pytest.mark.gpu

CONFIGS = {
    "cfg1": None,
    "cfg2": None,
    "cfg3": None,
    "small_free_noncommercial": dict(n_agents=2, n_cores=3, collection_length=3, priorities=[5], lengths=[5],
                                     probabilities=[1.0], free_prices=True, commercial=False),
    "two_jobs_per_round": dict(n_agents=3, n_cores=3, collection_length=4, priorities=[3, 10], lengths=[6, 3],
                               fix_prices=[2, 7], probabilities=[0.8, 0.2], new_jobs=2, reward_multiplier=2),
    "wide": dict(n_agents=21, n_cores=40, collection_length=6, priorities=[3, 10, 7], lengths=[6, 3, 2],
                 probabilities=[0.5, 0.3, 0.2], free_prices=True, commercial=True),
}


def _cfg(abi, name):
    kw = CONFIGS[name]
    return abi.named_config(name) if kw is None else abi.make_config(**kw)


def _compare_state(gs, os_list, E):
    for e in range(E):
        o = os_list[e]
        for k in ("round", "core_owner", "core_kind", "core_rem", "core_birth", "slot_kind", "slot_rem",
                  "slot_wait", "slot_birth", "offer_core", "offer_recip", "offer_price", "liab_n", "mt_index"):
            np.testing.assert_array_equal(gs[k][e], o[k], err_msg="%s env %d" % (k, e))
        np.testing.assert_array_equal(gs["mt"][e], o["mt"], err_msg="mt env %d" % e)
        for c in range(gs["liab_n"].shape[1]):
            n = gs["liab_n"][e, c]
            np.testing.assert_array_equal(gs["liab"][e, c, :n], o["liab"][c, :n])


@pytest.mark.parametrize("name", list(CONFIGS))
def test_step_bit_exact_vs_oracle(ms, oracle, name):
    abi = ms.abi
    cfg = _cfg(abi, name)
    s = abi.config_shape(cfg)
    N, C, L, O = s["N"], s["C"], s["L"], s["O"]
    E, T, seed = 24, 240, 7
    genv = ms.BatchedEnv(cfg, E, seed=seed)
    oenvs = [oracle.OracleEnv(cfg, seed + e) for e in range(E)]
    dev = genv.device
    obs = genv.reset(genv.obs_buffers(auctioneer=True))
    oobs = [o.observe() for o in oenvs]
    rng = np.random.default_rng(3)
    free = bool(cfg.free_prices)
    for t in range(T):
        acts = [random_actions(rng, offer_counts_from_obs(oobs[e]["acceptor"], O), N, C, L, O, free,
                               s["price_actions"] - 1, accept_bias=0.7) for e in range(E)]
        acc = torch.tensor(np.stack([a[0] for a in acts]), dtype=torch.int8, device=dev)
        off = torch.tensor(np.stack([a[1] for a in acts]), dtype=torch.int8, device=dev)
        pr = torch.tensor(np.stack([a[2] for a in acts]), dtype=torch.int8, device=dev) if free else None
        ev = genv.event_buffers()
        gobs, grew, gev = genv.step(acc, off, pr, obs=genv.obs_buffers(auctioneer=True), events=ev)
        ores = [oenvs[e].step(*acts[e]) for e in range(E)]
        oobs = [o.observe() for o in oenvs]
        ga = gobs["acceptor"].cpu().numpy()
        gof = gobs["offer"].cpu().numpy()
        gau = gobs["auctioneer"].cpu().numpy()
        for e in range(E):
            np.testing.assert_array_equal(ga[e, :, :, : s["acc_obs_dim"]], oobs[e]["acceptor"], err_msg="acc obs t=%d e=%d" % (t, e))
            assert (ga[e, :, :, s["acc_obs_dim"]:] == 0).all()
            np.testing.assert_array_equal(gof[e, :, :, : s["off_obs_dim"]], oobs[e]["offer"], err_msg="off obs t=%d e=%d" % (t, e))
            np.testing.assert_array_equal(gau[e, :, : s["acc_obs_dim"]], oobs[e]["auctioneer"], err_msg="auct obs t=%d" % t)
            np.testing.assert_array_equal(grew["acceptor"][e].cpu().numpy(), ores[e]["acceptor"], err_msg="acc rew t=%d e=%d" % (t, e))
            np.testing.assert_array_equal(grew["offer"][e].cpu().numpy(), ores[e]["offer"])
            if free:
                np.testing.assert_array_equal(grew["price"][e].cpu().numpy(), ores[e]["price"])
            np.testing.assert_array_equal(grew["auctioneer"][e].cpu().numpy(), ores[e]["auctioneer"])
            np.testing.assert_array_equal(grew["agent"][e].cpu().numpy(), ores[e]["agent"])
            gacc = ms.decode_accepted(gev["accepted"][e])
            gterm = ms.decode_terminated(gev["terminated"][e])
            for f in ("valid", "offerer", "recipient", "slot", "price", "nec_time", "prio", "kind", "order", "round"):
                np.testing.assert_array_equal(gacc[f][gacc["valid"] == 1], ores[e]["accepted"][f][ores[e]["accepted"]["valid"] == 1])
            np.testing.assert_array_equal(gacc["valid"], ores[e]["accepted"]["valid"])
            for f in ("valid", "owner", "prio", "init_len", "dwell"):
                np.testing.assert_array_equal(gterm[f], ores[e]["terminated"][f])
        if t % 40 == 0 or t == T - 1:
            _compare_state(genv.export_state(), [o.export_state() for o in oenvs], E)
    assert genv.flags() == 0
    assert genv.round == T


def test_separate_auctioneer_call_matches_oracle(ms, oracle):
    """ms_env_auctioneer (getAuctioneerAction before env.step, trainPPO.py:162) then ms_env_step with
    those actions: same actions, draws and state as the oracle's separate auctioneer call."""
    cfg = ms.abi.named_config("cfg3")
    s = ms.abi.config_shape(cfg)
    N, C, L, O = s["N"], s["C"], s["L"], s["O"]
    E, T, seed = 16, 120, 21
    genv = ms.BatchedEnv(cfg, E, seed=seed)
    oenvs = [oracle.OracleEnv(cfg, seed + e) for e in range(E)]
    dev = genv.device
    genv.reset()
    oobs = [o.observe() for o in oenvs]
    rng = np.random.default_rng(5)
    for t in range(T):
        acts = [random_actions(rng, offer_counts_from_obs(oobs[e]["acceptor"], O), N, C, L, O, True,
                               s["price_actions"] - 1, accept_bias=0.7) for e in range(E)]
        gauct = genv.auctioneer().cpu().numpy()
        oauct = [o.auctioneer_actions() for o in oenvs]
        for e in range(E):
            np.testing.assert_array_equal(gauct[e], oauct[e], err_msg="auct t=%d e=%d" % (t, e))
        acc = torch.tensor(np.stack([a[0] for a in acts]), dtype=torch.int8, device=dev)
        off = torch.tensor(np.stack([a[1] for a in acts]), dtype=torch.int8, device=dev)
        pr = torch.tensor(np.stack([a[2] for a in acts]), dtype=torch.int8, device=dev)
        genv.step(acc, off, pr, auctioneer=torch.tensor(gauct, dtype=torch.int8, device=dev))
        for e in range(E):
            oenvs[e].step(acts[e][0], acts[e][1], acts[e][2], np.asarray(oauct[e]))
        oobs = [o.observe() for o in oenvs]
        if t % 30 == 29:
            _compare_state(genv.export_state(), [o.export_state() for o in oenvs], E)
    # RNG state round trip (random.getstate()/setstate() words + index)
    words, idx = genv.get_rng_state(env_index=3)
    st = genv.export_state()
    assert list(words) == st["mt"][3].tolist() and idx == st["mt_index"][3]
    o = oracle.OracleEnv(cfg, 999)
    ost = o.export_state()
    genv.set_rng_state(ost["mt"].tolist(), int(ost["mt_index"]), env_index=3)
    assert [genv.randbelow(n, env_index=3) for n in (5, 9, 1000, 3)] == [o.randbelow(n) for n in (5, 9, 1000, 3)]


def test_randbelow_matches_oracle(ms, oracle):
    cfg = ms.abi.named_config("cfg2")
    genv = ms.BatchedEnv(cfg, 3, seed=11)
    o = oracle.OracleEnv(cfg, 12)
    ns = [1, 2, 3, 7, 8, 25, 97, 1000] * 100  # crosses several twists
    assert [genv.randbelow(n, env_index=1) for n in ns] == [o.randbelow(n) for n in ns]
    st = genv.export_state()
    ost = o.export_state()
    np.testing.assert_array_equal(st["mt"][1], ost["mt"])
    assert st["mt_index"][1] == ost["mt_index"]


def test_import_settlement_kat(ms):
    """round(7/6 * 105) = 123 (float64 product, half-even) on the device."""
    abi = ms.abi
    cfg = abi.make_config(2, 1, 1, priorities=[12], lengths=[6], probabilities=[1.0], free_prices=True)
    env = ms.BatchedEnv(cfg, 1, seed=0)
    st = env.export_state()
    st["round"][0] = 104
    st["core_owner"][0, 0] = 1
    st["core_kind"][0, 0] = 0
    st["core_rem"][0, 0] = 1
    st["core_birth"][0, 0] = 0
    st["liab_n"][0, 0] = 1
    st["liab"][0, 0, 0] = [1, 0, 7, 6, 0]
    st["slot_kind"][0, 0, 0] = 0  # agent 1 owns a core: keep >= 1 free slot? (L=1: slot must stay empty)
    st["slot_kind"][0, 0, 0] = -1
    env.import_state(st)
    d = env.device
    acc = torch.full((1, 2, 1), 2, dtype=torch.int8, device=d)
    off = torch.full((1, 2, 1), 1, dtype=torch.int8, device=d)
    pr = torch.full((1, 2, 1), -5, dtype=torch.int8, device=d)
    _, rew, _ = env.step(acc, off, pr, auctioneer=torch.full((1, 1), 2, dtype=torch.int8, device=d))
    assert int(rew["acceptor"][0, 0, 0]) == 12 - 123
    assert int(rew["agent"][0, 0]) == -123
    assert int(rew["auctioneer"][0, 0]) == 123


def test_full_size_cfg3_sampled_parity_and_determinism(ms, oracle):
    """BASELINE cfg3 size (16384 replicas): sampled envs bit-exact vs the oracle,
    and two runs with the same seed produce identical state (size-independent checks)."""
    abi = ms.abi
    cfg = abi.named_config("cfg3")
    s = abi.config_shape(cfg)
    E, T, seed = 16384, 60, 123
    sample = [0, 1, 4097, 9999, E - 1]
    gens = [ms.BatchedEnv(cfg, E, seed=seed) for _ in range(2)]
    oenvs = {e: oracle.OracleEnv(cfg, seed + e) for e in sample}
    d = gens[0].device
    g = torch.Generator(device=d)
    g.manual_seed(5)
    for t in range(T):
        acc = torch.randint(0, s["O"] + 1, (E, s["N"], s["C"]), generator=g, device=d, dtype=torch.int64)
        acc = torch.where(torch.rand(acc.shape, generator=g, device=d) < 0.7, torch.zeros_like(acc), acc).to(torch.int8)
        off = torch.randint(0, s["C"] + 1, (E, s["N"], s["L"]), generator=g, device=d).to(torch.int8)
        pr = torch.randint(0, s["price_actions"], (E, s["N"], s["L"]), generator=g, device=d).to(torch.int8)
        pr = torch.where(off == 0, torch.full_like(pr, -5), pr)
        outs = [ge.step(acc, off, pr) for ge in gens]
        a_np, o_np, p_np = acc.cpu().numpy(), off.cpu().numpy(), pr.cpu().numpy()
        ga = outs[0][0]["acceptor"].cpu().numpy()
        for e in sample:
            ores = oenvs[e].step(a_np[e], o_np[e], p_np[e])
            ob = oenvs[e].observe()
            np.testing.assert_array_equal(ga[e, :, :, : s["acc_obs_dim"]], ob["acceptor"])
            np.testing.assert_array_equal(outs[0][1]["acceptor"][e].cpu().numpy(), ores["acceptor"])
            np.testing.assert_array_equal(outs[0][1]["price"][e].cpu().numpy(), ores["price"])
        assert torch.equal(outs[0][0]["acceptor"], outs[1][0]["acceptor"])
        assert torch.equal(outs[0][1]["agent"], outs[1][1]["agent"])
    s0, s1 = gens[0].export_state(), gens[1].export_state()
    for k in s0:
        np.testing.assert_array_equal(s0[k], s1[k])
    for e in sample:
        ost = oenvs[e].export_state()
        np.testing.assert_array_equal(s0["mt"][e], ost["mt"])
        np.testing.assert_array_equal(s0["slot_kind"][e], ost["slot_kind"])
    assert gens[0].flags() == 0
