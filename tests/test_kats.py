"""Hand-derived known-answer scenarios (tests/golden/kats.json, made by tests/golden/make_kats.py)
run through the C oracle (CPU) and through ms_env_import + ms_env_step (GPU).

These are the only independent pin of the env semantics: the reference ships no fixtures and may
not be executed here, so every expectation in the fixture is written out by hand
from the reference text (file:line per scenario) with CPython's own `random` for the draws.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "kats.json")) as f:
    KATS = json.load(f)
IDS = [k["name"] for k in KATS]


def _cfg(abi, kat):
    return abi.make_config(**kat["config"])


def full_state(kat, cap):
    """Fixture state -> ms_state_host arrays for one env (liab: newest-first deque -> stored oldest first)."""
    st = {k: np.asarray(v, np.int32) for k, v in kat["state"].items() if k != "liab"}
    C = len(kat["state"]["core_owner"])
    liab = np.zeros((C, cap, 5), np.int32)
    liab_n = np.zeros(C, np.int32)
    for c, chain in enumerate(kat["state"]["liab"]):
        for q, entry in enumerate(reversed(chain)):
            liab[c, q] = entry
        liab_n[c] = len(chain)
    st.update(liab=liab, liab_n=liab_n, mt=np.asarray(kat["mt_words"], np.uint32),
              mt_index=np.int32(kat["mt_index"]), flags=np.uint32(0))
    return st


def check_state(got, exp, where):
    """got: exported state of one env (ms_state_host arrays); exp: the fixture's expected subset."""
    for k, v in exp.items():
        if k == "liab":
            for c, chain in enumerate(v):
                n = int(got["liab_n"][c])
                assert n == len(chain), "%s: liab_n[%d] %d != %d" % (where, c, n, len(chain))
                stored = np.asarray(got["liab"][c][:n])[::-1]  # newest first, as the reference's deque
                np.testing.assert_array_equal(stored.reshape(n, 5), np.asarray(chain, np.int32).reshape(n, 5),
                                              err_msg="%s liab core %d" % (where, c))
        else:
            np.testing.assert_array_equal(np.asarray(got[k]).reshape(np.shape(v)), np.asarray(v),
                                          err_msg="%s %s" % (where, k))


def check_obs(acc, off, auct, exp, s, where):
    if "acceptor" in exp:
        np.testing.assert_array_equal(np.asarray(acc)[..., : s["acc_obs_dim"]], exp["acceptor"], err_msg=where)
    if "offer" in exp:
        np.testing.assert_array_equal(np.asarray(off)[..., : s["off_obs_dim"]], exp["offer"], err_msg=where)
    if "auctioneer" in exp:
        np.testing.assert_array_equal(np.asarray(auct)[..., : s["acc_obs_dim"]], exp["auctioneer"], err_msg=where)


def check_rewards(got, exp, where):
    for k, v in exp.items():
        np.testing.assert_array_equal(np.asarray(got[k]).reshape(np.shape(v)), np.asarray(v), err_msg="%s %s" % (where, k))


def test_kat_fixture_is_current():
    """The committed fixture equals what the generator writes (no hand edits drift)."""
    import subprocess
    import sys
    import tempfile

    gen = os.path.join(HERE, "golden", "make_kats.py")
    with tempfile.TemporaryDirectory() as d:
        src = open(gen).read().replace('HERE = os.path.dirname(os.path.abspath(__file__))', 'HERE = %r' % d)
        p = os.path.join(d, "gen.py")
        open(p, "w").write(src)
        subprocess.check_call([sys.executable, p], stdout=subprocess.DEVNULL)
        assert json.load(open(os.path.join(d, "kats.json"))) == KATS


@pytest.mark.parametrize("kat", KATS, ids=IDS)
def test_kat_oracle(oracle, kat):
    cfg = _cfg(oracle.abi, kat)
    s = oracle.abi.config_shape(cfg)
    if kat.get("device_only"):
        pytest.skip(kat["device_only"])
    env = oracle.OracleEnv(cfg, 0)
    env.import_state(full_state(kat, s["liability_cap"]))
    for i, step in enumerate(kat["steps"]):
        where = "%s step %d (oracle)" % (kat["name"], i)
        exp = step["expect"]
        if "error" in exp:  # the device refuses the round (MS_EOVERFLOW); the oracle keeps its flags
            assert env.flags & 0x01, where
            continue
        r = env.step(step["acc"], step["off"], step["price"], step["auct"])
        got = env.export_state()
        check_state(got, exp.get("state", {}), where)
        if exp.get("mt_index") is not None:
            assert int(got["mt_index"]) == exp["mt_index"], where
        ob = env.observe()
        check_obs(ob["acceptor"], ob["offer"], ob["auctioneer"], exp.get("obs", {}), s, where)
        check_rewards(r, exp.get("rewards", {}), where)
        if "termination_revenue" in exp:
            assert r["termination_revenue"] == exp["termination_revenue"], where
        if "flags_set" in exp:
            assert env.flags & exp["flags_set"] == exp["flags_set"], where
        else:
            assert env.flags == 0, where


@pytest.mark.gpu
@pytest.mark.parametrize("kat", KATS, ids=IDS)
def test_kat_device(ms, kat):
    import torch

    cfg = _cfg(ms.abi, kat)
    s = ms.abi.config_shape(cfg)
    env = ms.BatchedEnv(cfg, 1, seed=0)
    env.import_state({k: np.asarray(v)[None] for k, v in full_state(kat, env.shape.liability_cap).items()})
    d = env.device
    N, C, L = s["N"], s["C"], s["L"]
    for i, step in enumerate(kat["steps"]):
        where = "%s step %d (device)" % (kat["name"], i)
        t8 = lambda x, shape: torch.tensor(np.asarray(x, np.int64).reshape(shape), dtype=torch.int8, device=d)
        # acc = off = None: the hard-coded agents act inside the round (ms_actions.acceptor = offer_core = NULL)
        acc = t8(step["acc"], (1, N, C)) if step["acc"] is not None else None
        off = t8(step["off"], (1, N, L)) if step["off"] is not None else None
        pr = t8(step["price"], (1, N, L)) if step["price"] is not None else None
        auct = t8(step["auct"], (1, C)) if step["auct"] is not None else None
        exp = step["expect"]
        if "error" in exp:
            with pytest.raises(ms.MarlSchedError) as ei:
                env.step(acc, off, pr, auctioneer=auct, obs=env.obs_buffers(auctioneer=True))
            assert ei.value.code == exp["error"], where
            continue
        obs, rew, _ = env.step(acc, off, pr, auctioneer=auct, obs=env.obs_buffers(auctioneer=True))
        got = {k: v[0] for k, v in env.export_state().items()}
        check_state(got, exp.get("state", {}), where)
        if exp.get("mt_index") is not None:
            assert int(got["mt_index"]) == exp["mt_index"], where
        check_obs(obs["acceptor"][0].cpu(), obs["offer"][0].cpu(), obs["auctioneer"][0].cpu(), exp.get("obs", {}), s,
                  where)
        check_rewards({k: v[0].cpu().numpy() for k, v in rew.items() if v is not None}, exp.get("rewards", {}), where)
        if "flags_set" in exp:
            assert int(got["flags"]) & exp["flags_set"] == exp["flags_set"], where
        else:
            assert int(got["flags"]) == 0, where
