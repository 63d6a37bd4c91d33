"""The locally shared free-price rollout in one launch (ms_env_rollout_act_free, k_env_rollout_act_free; ABI 17).

BASELINE cfg3 (8 agents x 8 cores, free prices + commercial reward, locally shared PPO) used to run every round
as two launches: the paired act kernel (k_act_pair<1,1,1,2,2>: core + price choosers and compact acceptors,
SchedulingEnvironment.py:150-172) and the env round (k_env_step, world.py:295-334). The one-launch rollout steps
a workgroup's 4 N replicas (16 lanes each) and then acts for them with one wave per agent from the observations
still in its LDS, round after round. It must change nothing: every ring (observations, actions, log-probs,
rewards, price states), every loss and weight, and the env state after the rollout equal the two-launch
trainer's bit for bit, over two PPO iterations (the second acting on updated nets: act fragments, price table
and common-row tables rebuilt)."""
import importlib

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rings(t):
    out = {"acc_rows": t.acc_rows, "acc_owner": t.acc_owner, "off_obs": t.off_obs, "env_price": t.env_price,
           "agent_reward": t.agent_reward, "auct_reward": t.auct_reward}
    if t.price_obs is not None:
        out["price_obs"] = t.price_obs
    for u in t.units():
        for k in ("actions", "logprobs", "rewards"):
            out["%s.%s" % (u.name, k)] = getattr(u, k)
    return out


def _trainers(monkeypatch, mk):
    fused = mk()
    monkeypatch.setenv("MS_ENV_ROLLOUT_FREE", "0")
    plain = mk()
    monkeypatch.delenv("MS_ENV_ROLLOUT_FREE")
    assert fused.fused_rollout_free and not plain.fused_rollout_free
    return fused, plain


def _compare(trs, iters=2):
    for it in range(iters):
        for t in trs:
            t.rollout()
        torch.cuda.synchronize()
        r0, r1 = _rings(trs[0]), _rings(trs[1])
        for k in r0:
            same = r0[k] == r1[k]
            assert bool(same.all()), (it, k, int((~same).sum()), same.numel())
        losses = [t.update() for t in trs]
        for k in losses[0]:
            assert torch.equal(losses[0][k], losses[1][k]), (it, k)
    ppo = importlib.import_module("marl-scheduling_amd.ppo")
    for u0, u1 in zip(trs[0].units(), trs[1].units()):
        for k in ppo.ACTOR_KEYS + ppo.CRITIC_KEYS:
            assert torch.equal(getattr(u0.group.policy, k), getattr(u1.group.policy, k)), (u0.name, k)
    assert all(t.flags() == 0 for t in trs)
    st = [t.env.parts[0][0].export_state() for t in trs]
    for k in st[0]:
        assert (st[0][k] == st[1][k]).all(), k


@pytest.mark.parametrize("E,T,own", [(16384, 200, "1"), (2048, 16, "1"), (2048, 16, "0"), (1001, 12, "1")])
def test_cfg3_one_launch_rollout_equals_two_launches(ms, monkeypatch, E, T, own):
    """cfg3 at the BASELINE size (E 16384, UPDATE_STEP 200: every replica crosses MT blocks inside the launch),
    at E 2048 and at E 1001 (a last workgroup of 9 replicas: 4 N = 32 per workgroup), the FixShape<8,8,3,1>
    kernel: equal to the act launch + env launch per round, bit for bit. own "1": the owned acceptor items go
    through the by-core buffers (ABI 18) and the fill writes whole rows; "0": straight into the rings."""
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    monkeypatch.setenv("MS_FILL_OWN", own)
    trs = _trainers(monkeypatch, lambda: tr_mod.Trainer.from_named("cfg3", n_envs=E, update_step=T, seed=11,
                                                                    device="cuda:0"))
    assert (trs[0].acc_own is not None) == (own == "1")
    _compare(trs)


@pytest.mark.parametrize("N,C,L,E", [(6, 6, 3, 500), (8, 7, 2, 256), (4, 9, 4, 130)])
def test_generic_shape_one_launch_rollout_equals_two_launches(ms, monkeypatch, N, C, L, E):
    """Other locally shared free-price shapes run the DynShape kernel (6 x 6 x 3: 6 waves per workgroup;
    8 x 7 x 2: 2C = 14, the slot pair inside a template dword; 4 x 9 x 4: 144 acceptor items per workgroup, so
    the 64-item draw pairing is not aligned to the workgroups): equal to the two launches."""
    abi = importlib.import_module("marl-scheduling_amd.abi")
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    cfg = abi.make_config(N, C, L, free_prices=True, commercial=True, **abi.EXP4_JOBS)
    hp = tr_mod.Hyper(update_step=10, raw_k_epochs=2)
    trs = _trainers(monkeypatch, lambda: tr_mod.Trainer(cfg, E, arch="local", hyper=hp, seed=4, device="cuda:0"))
    _compare(trs)


def test_cfg3_one_launch_rollout_of_parts(ms, monkeypatch):
    """Two rollout streams (two replica parts, each its own env and launch, rows from their global replica
    index): equal to the single two-launch trainer, bit for bit."""
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    mk = lambda streams: tr_mod.Trainer.from_named("cfg3", n_envs=512, update_step=12, seed=7, device="cuda:0",
                                                   rollout_streams=streams)
    parts = mk(2)
    monkeypatch.setenv("MS_ENV_ROLLOUT_FREE", "0")
    plain = mk(1)
    assert parts.fused_rollout_free and not plain.fused_rollout_free
    for it in range(2):
        for t in (parts, plain):
            t.rollout()
        torch.cuda.synchronize()
        r0, r1 = _rings(parts), _rings(plain)
        for k in r0:
            assert torch.equal(r0[k], r1[k]), (it, k)
        l0, l1 = parts.update(), plain.update()
        for k in l0:
            assert torch.equal(l0[k], l1[k]), (it, k)


def test_rollout_act_free_rejects_unsupported_calls(ms):
    """ms_env_rollout_act_free's argument checks (include/marlsched.h): n_rounds >= 1, a price table, act
    fragments, offer_price = the acting's env_price buffer, no event records, a supported env; each refusal is
    MS_EINVAL with a message and leaves the env's round counter where it was. A ring shorter than n_rounds slots
    is refused on the host (BatchedEnv.check_rings) before any launch."""
    lib_mod = importlib.import_module("marl-scheduling_amd._lib")
    abi = importlib.import_module("marl-scheduling_amd.abi")
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    t = tr_mod.Trainer.from_named("cfg3", n_envs=64, update_step=8, seed=2, device="cuda:0")
    assert t.fused_rollout_free
    t._prepare_acting()
    env, e0, e1 = t.env.parts[0]
    E, N, C, L = e1 - e0, t.N, t.C, t.L
    obs = dict(t._acc_out(1, e0, e1), offer=t.off_obs[1])
    rew = dict(offer=t.off.rewards[0].view(E, N, L), acceptor=t.acc.rewards[0].view(E, N, C), agent=t.agent_reward,
               auctioneer=t.auct_reward, price=t.price.rewards[0].view(E, N, L))
    strides = abi.MsRoundStridesFree(*([0] * 17 + [8]))
    nxt, out = t._fused_next_free(1, 0)
    acc0, off0 = t.acc.actions[0].view(E, N, C), t.off.actions[0].view(E, N, L)
    r0 = lib_mod.lib.ms_env_round(env._h)
    with pytest.raises(lib_mod.MarlSchedError, match="n_rounds"):
        env.rollout_act_free(acc0, off0, obs, rew, nxt, out, strides, 0)
    with pytest.raises(lib_mod.MarlSchedError, match="event records"):
        env.rollout_act_free(acc0, off0, obs, rew, nxt, out, strides, 1,
                             events=dict(accepted=torch.zeros((E, C, 16), dtype=torch.uint8, device="cuda:0")))
    bad = abi.MsFusedActFree.from_buffer_copy(nxt)
    bad.price_table = None
    with pytest.raises(lib_mod.MarlSchedError, match="price table"):
        env.rollout_act_free(acc0, off0, obs, rew, bad, out, strides, 1)
    bad = abi.MsFusedActFree.from_buffer_copy(nxt)
    bad.acceptor.act_frag = None
    with pytest.raises(lib_mod.MarlSchedError, match="act fragments"):
        env.rollout_act_free(acc0, off0, obs, rew, bad, out, strides, 1)
    assert lib_mod.lib.ms_env_round(env._h) == r0
    # a ring of T slots asked for T + 1 rounds at its stride
    b = lambda x: x.stride(0) * x.element_size()
    long = abi.MsRoundStridesFree(b(t.acc.actions), b(t.off.actions), b(t.acc_rows), b(t.acc_owner), b(t.off_obs),
                                  b(t.off.rewards), b(t.price.rewards), b(t.acc.rewards), 0, 0, b(t.off.actions),
                                  b(t.off.logprobs), b(t.price_obs), b(t.price.actions), b(t.price.logprobs),
                                  b(t.acc.actions), b(t.acc.logprobs), 8)
    with pytest.raises(AssertionError, match="n_rounds slots"):
        env.rollout_act_free(acc0, off0, obs, rew, nxt, out, long, t.T + 1)
    assert lib_mod.lib.ms_env_round(env._h) == r0
    fixed = tr_mod.Trainer.from_named("cfg2", n_envs=64, update_step=8, seed=2, device="cuda:0")
    assert not fixed.fused_rollout_free and not fixed.env.parts[0][0].rollout_free_supported()


@pytest.mark.parametrize("name", ["cfg2", "cfg3"])
def test_one_round_rollouts(ms, name):
    """UPDATE_STEP 1: the fused rollouts write round t + 1's acting into ring slot t + 1, which a
    one-slot ring does not have, so they are off and the trainer runs the per-round launches."""
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    t = tr_mod.Trainer.from_named(name, n_envs=64, update_step=1, seed=1, device="cuda:0")
    assert not t.fused_rollout and not t.fused_rollout_free
    for _ in range(2):
        t.iteration()
    torch.cuda.synchronize()
    assert t.flags() == 0 and t.rounds_done == 2


@pytest.mark.parametrize("name,E", [("cfg3", 2048), ("cfg2", 1024), ("cfg4", 256)])
def test_update_streams_equal_one_stream(ms, monkeypatch, name, E):
    """One rank updates each unit type on its own stream by default (Trainer.update_streams; the unit types are
    independent nets, PPOmodules.py:548-597): every loss and weight equals the one-stream update's bit for bit,
    over three iterations (each acting on the previous update's weights), graph-replayed. cfg3's trainer with
    streams also defers (MS_DEFER_COMMON=1) the rollout's common acceptor items into the update: every ring equals the
    one-stream trainer's after each iteration."""
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    ppo = importlib.import_module("marl-scheduling_amd.ppo")
    mk = lambda: tr_mod.Trainer.from_named(name, n_envs=E, update_step=12, seed=6, device="cuda:0")
    monkeypatch.setenv("MS_DEFER_COMMON", "1")
    streams = mk()
    monkeypatch.setenv("MS_UPDATE_STREAMS", "0")
    one = mk()
    assert streams.update_streams and not one.update_streams
    assert streams.defer_common == (name == "cfg3") and not one.defer_common
    for it in range(3):
        l0, l1 = streams.iteration(), one.iteration()
        torch.cuda.synchronize()
        for k in l0:
            assert torch.equal(l0[k], l1[k]), (it, k)
        r0, r1 = _rings(streams), _rings(one)
        for k in r0:
            assert torch.equal(r0[k], r1[k]), (it, k)
    for u0, u1 in zip(streams.units(), one.units()):
        for k in ppo.ACTOR_KEYS + ppo.CRITIC_KEYS:
            assert torch.equal(getattr(u0.group.policy, k), getattr(u1.group.policy, k)), (u0.name, k)
