"""Compact acceptor observations at every env-round launch variant the trainers ship (VERDICT r4 missing 2).

launch_env_step (env_kernels.hip) picks the lanes per replica from the replica count and a kernel
compiled for the BASELINE shape or the generic one, and the trainers run the compact variant
(k_env_step<LPE, false, true, SH>: owner rows + owners instead of the N*C acceptor rows). Each case
below is one variant the trainers run:

  cfg2 E=4096   LPE 32  FixShape<4,4,3,1>  (the cfg2 bench line's kernel)
  cfg3 E=2048   LPE 64  DynShape           (lanes widened to reach 2048 waves)
  cfg3 E=4096   LPE 32  DynShape
  cfg3 E=16384  LPE 16  FixShape<8,8,3,1>  (the headline kernel)

For each: the compact trainer == the materialised trainer (k_env_step<LPE, false, false, SH> and the
row-reading act / gradient kernels) bit for bit over two PPO iterations (every ring, loss and weight),
and three replicas of the compact trainer's first rollout replayed through the C oracle with the
actions its rings hold (world.py:295-334; observations and rewards bit-exact)."""
import importlib

import pytest
import torch

from tests.replay import oracle_replay

pytestmark = pytest.mark.gpu

CASES = [("cfg2", 4096, 16), ("cfg3", 2048, 16), ("cfg3", 4096, 16), ("cfg3", 16384, 12)]


def _rings(t):
    out = {"acceptor_rows": t.acceptor_rows(), "off_obs": t.off_obs}
    if t.price_obs is not None:
        out["price_obs"] = t.price_obs
    for u in t.units():
        for k in ("actions", "logprobs", "rewards"):
            out["%s.%s" % (u.name, k)] = getattr(u, k)
    return out


@pytest.mark.parametrize("name,E,T", CASES)
def test_compact_trainer_equals_materialised_and_oracle(ms, name, E, T):
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    ppo = importlib.import_module("marl-scheduling_amd.ppo")
    seed = 5
    trs = [tr_mod.Trainer.from_named(name, n_envs=E, update_step=T, seed=seed, device="cuda:0", compact=c)
           for c in (True, False)]
    assert trs[0].compact and not trs[1].compact
    for it in range(2):
        for t in trs:
            t.rollout()
        torch.cuda.synchronize()
        r0, r1 = _rings(trs[0]), _rings(trs[1])
        for k in r0:
            assert torch.equal(r0[k], r1[k]), (it, k)
        if it == 0:
            oracle_replay(trs[0], (0, E // 2 + 1, E - 1), tr_mod.env_seed(seed, 0, E), T)
        losses = [t.update() for t in trs]
        for k in losses[0]:
            assert torch.equal(losses[0][k], losses[1][k]), (it, k)
    for u0, u1 in zip(trs[0].units(), trs[1].units()):
        for k in ppo.ACTOR_KEYS + ppo.CRITIC_KEYS:
            assert torch.equal(getattr(u0.group.policy, k), getattr(u1.group.policy, k)), (u0.name, k)
    assert all(t.flags() == 0 for t in trs)


@pytest.mark.parametrize("E,T", [(4096, 16), (4096, 200), (96, 24), (1001, 12)])
def test_fused_env_act_equals_two_launches(ms, monkeypatch, E, T):
    """cfg2 (fixed prices, one net per role): round t's env launch also samples round t + 1's actions from
    the observations in its LDS (ms_env_step_act), and by default the whole rollout is one launch
    (ms_env_rollout_act: each wave loops over the rounds). Every ring of the one-launch rollout, of the
    launch-per-round rollout and of the two-launch trainer (the paired act launch, then the env launch)
    are equal bit for bit over two iterations: E = 4096 runs k_env_*_act<32, FixShape<4,4,3,1>> (T = 200: the
    BASELINE rollout length, every env crossing MT blocks inside the one launch), E = 96
    the LPE-16 generic one (four replicas per wave), E = 1001 a partial last wave (one replica)."""
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    mk = lambda: tr_mod.Trainer.from_named("cfg2", n_envs=E, update_step=T, seed=9, device="cuda:0")
    whole = mk()
    monkeypatch.setenv("MS_ENV_ROLLOUT", "0")
    per_round = mk()
    monkeypatch.setenv("MS_ENV_FUSED_ACT", "0")
    plain = mk()
    assert whole.fused_rollout and per_round.fused_step and not per_round.fused_rollout and not plain.fused_step
    trs = (whole, per_round, plain)
    for it in range(2):
        for t in trs:
            t.rollout()
        torch.cuda.synchronize()
        rings = [_rings(t) for t in trs]
        for k in rings[0]:
            for r in rings[1:]:
                assert torch.equal(rings[0][k], r[k]), (it, k)
        losses = [t.update() for t in trs]
        for k in losses[0]:
            for l in losses[1:]:
                assert torch.equal(losses[0][k], l[k]), (it, k)
    assert all(t.flags() == 0 for t in trs)
    # the env state after the rollouts too (ms_env_export)
    st = [t.env.parts[0][0].export_state() for t in trs]
    for k in st[0]:
        for o in st[1:]:
            assert (st[0][k] == o[k]).all(), k


def test_rollout_act_rejects_unsupported_calls(ms):
    """ms_env_rollout_act's argument checks (include/marlsched.h): n_rounds >= 1, no accepted /
    terminated event records, a fixed-price env; each refusal is MS_EINVAL with a message, and the
    env is left as it was (its round counter does not move)."""
    lib_mod = importlib.import_module("marl-scheduling_amd._lib")
    abi = importlib.import_module("marl-scheduling_amd.abi")
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    t = tr_mod.Trainer.from_named("cfg2", n_envs=96, update_step=8, seed=2, device="cuda:0")
    assert t.fused_rollout
    env, e0, e1 = t.env.parts[0]
    E, N, C, L = e1 - e0, t.N, t.C, t.L
    obs = dict(t._acc_out(1, e0, e1), offer=t.off_obs[1])
    rew = dict(offer=t.off.rewards[0].view(E, N, L), acceptor=t.acc.rewards[0].view(E, N, C), agent=t.agent_reward,
               auctioneer=t.auct_reward)
    strides = abi.MsRoundStrides(*([0] * 13 + [8]))
    nxt = t._fused_next(1, 0)
    acc0, off0 = t.acc.actions[0].view(E, N, C), t.off.actions[0].view(E, N, L)
    r0 = lib_mod.lib.ms_env_round(env._h)
    with pytest.raises(lib_mod.MarlSchedError, match="n_rounds"):
        env.rollout_act(acc0, off0, obs, rew, nxt, strides, 0)
    acc_ev = torch.zeros((E, C, 16), dtype=torch.uint8, device="cuda:0")
    with pytest.raises(lib_mod.MarlSchedError, match="event records"):
        env.rollout_act(acc0, off0, obs, rew, nxt, strides, 1, events=dict(accepted=acc_ev))
    assert lib_mod.lib.ms_env_round(env._h) == r0
    free = tr_mod.Trainer.from_named("cfg3", n_envs=64, update_step=8, seed=2, device="cuda:0")
    assert not free.fused_rollout and not free.env.parts[0][0].fused_act_supported()
