"""The trainers at their per-GPU BASELINE sizes ("test the untested configs").

* cfg3 (16384 x 8 x 8, locally shared free-price PPO, T = 200): one full iteration. The update's
  per-draw losses of sampled agents are recomputed by the torch restatement of the reference's
  ``LocallySharedPPO.update`` (oracle/ppo_ref.RefPPO: PPOmodules.py:548-597, the same optimizer
  across the draws) on that agent's sub-unit rows of every replica, read from the trainer's own
  rollout rings, with the pre-update weights.
* cfg4 (8192 x 16 x 16, divided free-price PPO, K = 3): one iteration, finite losses, no env
  flags, a same-seed repeat bit-identical, two replicas' trajectories replayed through the C
  oracle from the trainer's action rings, and one divided acceptor unit's 3 epochs vs RefPPO.
* cfg5 (8192 x 32 x 32, Branching DQN): a few frames, finite losses, no flags, and two replicas'
  trajectories vs the C oracle from the trainer's action ring.

Returns are per replica (E = 1 semantics of PPOmodules.py:548-560), rows r = t * E + e.
Tolerances: the first draw's loss 1e-5 relative (north star); after an Adam step the weights
agree within 1e-4 relative (Adam divides by sqrt(v), which amplifies last-ulp gradient order
differences), so later draws' losses are held to 1e-4."""
import importlib
import random

import numpy as np
import pytest
import torch

from oracle import pyoracle
from oracle.ppo_ref import RefPPO

pytestmark = pytest.mark.gpu


def _tr():
    return importlib.import_module("marl-scheduling_amd.trainer")


def _ppo():
    return importlib.import_module("marl-scheduling_amd.ppo")


def _returns(rewards_te, gamma):
    """PPOmodules.py:548-560 per replica: float64 Monte-Carlo returns (Python float arithmetic ==
    float64), cast to float32, normalised with the unbiased std: [T, E] -> [T * E] rows t * E + e."""
    r = rewards_te.double().cpu()
    T = r.shape[0]
    out = torch.empty_like(r)
    g = torch.zeros(r.shape[1], dtype=torch.float64)
    for t in range(T - 1, -1, -1):
        g = r[t] + gamma * g
        out[t] = g
    f = out.float()
    f = (f - f.mean(0, keepdim=True)) / (f.std(0, keepdim=True) + 1e-7)
    return f.reshape(-1)


def _ref_from_group(grp, g, D, A, hp):
    """A RefPPO whose policy holds group g's current weights (on the device)."""
    ppo = _ppo()
    ref = RefPPO(D, A, hp.lr_actor, hp.lr_critic, grp.gamma, hp.eps_clip, grp.K)
    with torch.no_grad():
        for k, v in ref.policy.flat().items():
            v.copy_(getattr(grp.policy, k)[g].detach().cpu())
    assert set(ref.policy.flat()) == set(ppo.ACTOR_KEYS + ppo.CRITIC_KEYS)
    ref.policy.cuda()
    ref.policy_old.cuda()
    return ref


def _unit_rows(tr, u, unit, T):
    """(states [T*E, D] float, actions [T*E], old log-probs [T*E], rewards [T, E]) of one unit."""
    if u is tr.acc:
        own = tr.acc_owner[:T, :, unit % tr.C]
        a = unit // tr.C
        rows = torch.where((own == a + 1).unsqueeze(-1), tr.acc_rows[:T, :, unit % tr.C], tr.acc_common)
    elif u is tr.off:
        rows = tr.off_obs[:T, :, unit]
    else:
        rows = tr.price_obs[:T, :, unit]
    x = rows[..., : u.D].reshape(-1, u.D).float()
    return (x, u.actions[:, :, unit].reshape(-1).long(), u.logprobs[:, :, unit].reshape(-1).float(),
            u.rewards[:, :, unit])


def _weights_close(got, want, lr, steps, what):
    """Weights after Adam steps: within 1e-4 relative / 1e-5 absolute except for the few elements
    whose gradient is a near-cancellation of millions of rows (its sign is then last-ulp noise, and
    Adam's normalised step m / sqrt(v) turns either sign into a full +-lr step): at most 1 % of the
    elements may differ more, and none by more than the 2 lr a step can move them apart."""
    d = (got - want).abs()
    loose = d > 1e-5 + 1e-4 * want.abs()
    assert loose.float().mean().item() <= 0.01, (what, int(loose.sum()), d.max().item())
    assert d.max().item() <= 2 * lr * steps + 1e-6, (what, d.max().item())


def _local_draws(rng_state, N, C, L, CS):
    """Trainer._draws for the locally shared arch (Agent.py:716-728) from a saved random state."""
    rng = random.Random()
    rng.setstate(rng_state)
    acc = [[0] * N for _ in range(CS)]
    off = [[0] * N for _ in range(CS)]
    for a in range(N):
        for i in range(CS):
            acc[i][a] = a * C + rng.randint(0, C - 1)
        for j in range(CS):
            off[j][a] = a * L + rng.randint(0, L - 1)
    return dict(acceptor=acc, offer=off, price=off)


def test_cfg3_fullsize_iteration_losses_match_refppo(ms):
    tr = _tr().Trainer.from_named("cfg3", seed=7, device="cuda:0")
    assert tr.E == 16384 and tr.T == 200
    tr.rollout()
    torch.cuda.synchronize()
    assert tr.flags() == 0
    T = tr.T
    agents = (0, 5)
    refs = {u.name: {a: _ref_from_group(u.group, a, u.D, u.group.policy.A, tr.hp) for a in agents}
            for u in tr.units()}
    draws = _local_draws(tr.rng.getstate(), tr.N, tr.C, tr.L, tr.hp.centralisation_sample)
    # the update ends by carrying ring slot T into slot 0 (the next iteration's first observation):
    # keep slot 0 as the update saw it for the reference rows
    slot0 = [x[0].clone() for x in (tr.acc_rows, tr.acc_owner, tr.off_obs)]
    losses = tr.update()
    torch.cuda.synchronize()
    for x, s0 in zip((tr.acc_rows, tr.acc_owner, tr.off_obs), slot0):
        x[0].copy_(s0)
    for u in tr.units():
        got = losses[u.name].cpu().numpy()            # [steps = draws x K, G]
        K = u.group.K
        assert got.shape == (len(draws[u.name]) * K, tr.N)
        assert np.isfinite(got).all()
        for a in agents:
            ref = refs[u.name][a]
            want = []
            for d, sel in enumerate(draws[u.name]):
                x, act, lp, rw = _unit_rows(tr, u, sel[a], T)
                want += ref.update(x, act, lp, _returns(rw, u.group.gamma).cuda())
            for s, w in enumerate(want):
                rtol = 1e-5 if s < K else 1e-4
                np.testing.assert_allclose(got[s, a], w, rtol=rtol, atol=1e-6, err_msg="%s agent %d step %d"
                                           % (u.name, a, s))
            steps = len(want)
            for k, v in ref.policy.flat().items():
                _weights_close(getattr(u.group.policy, k)[a].detach().cpu(), v.detach().cpu(),
                               tr.hp.lr_critic if k.startswith("c") else tr.hp.lr_actor, steps,
                               "%s agent %d %s" % (u.name, a, k))


def _oracle_replay(tr, replicas, base_seed, T):
    """Step the C oracle of replicas e with the actions the trainer's rings hold and compare its
    observations and rewards with the rings (slot t + 1 = the observation after round t)."""
    cfg = tr.cfg
    s = pyoracle.abi.config_shape(cfg)
    N, C, L, D_acc, D_off = s["N"], s["C"], s["L"], s["acc_obs_dim"], s["off_obs_dim"]
    idx = torch.tensor(list(replicas), device=tr.acc_rows.device)
    acc_all = _ppo().regen_acceptor_rows(tr.acc_rows.index_select(1, idx).contiguous(),
                                         tr.acc_owner.index_select(1, idx).contiguous(), tr.acc_common,
                                         tr.N).cpu().numpy()                # [T+1, n, N*C, stride]
    off_all = tr.off_obs[:, list(replicas)].cpu().numpy()
    aa = tr.acc.actions[:, list(replicas)].cpu().numpy()
    ao = tr.off.actions[:, list(replicas)].cpu().numpy()
    ap = tr.price.actions[:, list(replicas)].cpu().numpy() if tr.free else None
    ra = tr.acc.rewards[:, list(replicas)].cpu().numpy()
    ro = tr.off.rewards[:, list(replicas)].cpu().numpy()
    rp = tr.price.rewards[:, list(replicas)].cpu().numpy() if tr.free else None
    for i, e in enumerate(replicas):
        env = pyoracle.OracleEnv(cfg, base_seed + e)
        o = env.observe()
        assert np.array_equal(acc_all[0, i, :, :D_acc].reshape(N, C, D_acc), o["acceptor"]), e
        for t in range(T):
            core = ao[t, i].reshape(N, L)
            price = np.where(core == 0, -5, ap[t, i].reshape(N, L)) if tr.free else None
            r = env.step(aa[t, i].reshape(N, C), core, price)
            o = env.observe()
            assert np.array_equal(acc_all[t + 1, i, :, :D_acc].reshape(N, C, D_acc), o["acceptor"]), (e, t)
            assert np.array_equal(off_all[t + 1, i, :, :D_off].reshape(N, L, D_off), o["offer"]), (e, t)
            assert np.array_equal(ra[t, i].reshape(N, C), r["acceptor"]), (e, t)
            assert np.array_equal(ro[t, i].reshape(N, L), r["offer"]), (e, t)
            if tr.free:
                assert np.array_equal(rp[t, i].reshape(N, L), r["price"]), (e, t)


def _cfg4_run(seed):
    tr = _tr().Trainer.from_named("cfg4", n_envs=8192, seed=seed, device="cuda:0")
    assert tr.arch == "divided" and tr.E == 8192 and tr.N == 16 and tr.C == 16
    return tr


def test_cfg4_fullsize_iteration(ms):
    tr = _cfg4_run(11)
    T = tr.T
    tr.rollout()
    torch.cuda.synchronize()
    assert tr.flags() == 0
    # divided: every unit its own net; check acceptor unit 37 (agent 2, core 5) over its K epochs
    unit = 37
    u = tr.acc
    ref = _ref_from_group(u.group, unit, u.D, u.group.policy.A, tr.hp)
    x, act, lp, rw = _unit_rows(tr, u, unit, T)
    want = ref.update(x, act, lp, _returns(rw, u.group.gamma).cuda())
    _oracle_replay(tr, (0, 8191), _tr().env_seed(11, 0, 8192), T)
    losses = tr.update()
    torch.cuda.synchronize()
    for k, v in losses.items():
        assert torch.isfinite(v).all(), k
    got = losses["acceptor"][:, unit].cpu().numpy()
    assert got.shape == (u.group.K,)
    for s, w in enumerate(want):
        np.testing.assert_allclose(got[s], w, rtol=1e-5 if s == 0 else 1e-4, atol=1e-6, err_msg="epoch %d" % s)
    keep = {k: v.cpu() for k, v in losses.items()}
    weights = {(un.name, k): getattr(un.group.policy, k).detach().cpu().clone() for un in tr.units()
               for k in _ppo().ACTOR_KEYS + _ppo().CRITIC_KEYS}
    obs = tr.off_obs.cpu().clone()
    del tr
    torch.cuda.empty_cache()
    # the same seed again: bit-identical losses, weights and rollout
    tr2 = _cfg4_run(11)
    tr2.rollout()
    losses2 = tr2.update()
    torch.cuda.synchronize()
    for un in tr2.units():
        for k in _ppo().ACTOR_KEYS + _ppo().CRITIC_KEYS:
            assert torch.equal(getattr(un.group.policy, k).detach().cpu(), weights[(un.name, k)]), (un.name, k)
    assert torch.equal(tr2.off_obs.cpu(), obs)
    for k in keep:
        assert torch.equal(keep[k], losses2[k].cpu()), k


def test_cfg5_fullsize_frames(ms):
    bdqn = importlib.import_module("marl-scheduling_amd.bdqn")
    abi = importlib.import_module("marl-scheduling_amd.abi")
    cfg = abi.named_config("cfg5")
    E, frames, seed = 8192, 6, 3
    tr = bdqn.BDQNTrainer(cfg, n_envs=E, bcfg=bdqn.BDQNConfig(memory_frames=16, learning_starts=2), seed=seed,
                          device="cuda:0")
    assert tr.N == 32 and tr.C == 32
    N, C, L = tr.N, tr.C, tr.L
    picks = (0, E - 1)
    acts = []
    for f in range(frames):
        slot = tr.head
        tr.step()
        acts.append({k: v[slot][list(picks)].cpu().numpy() for k, v in tr.act.items()})
    torch.cuda.synchronize()
    assert tr.flags() == 0
    assert set(tr.last_losses) >= {"acc", "off"}
    assert all(torch.isfinite(v).all() for v in tr.last_losses.values())
    # the oracle replays replicas 0 and E-1 with the actions the trainer took; the final state's
    # compact observation (ring slot head) must equal the oracle's observation
    s = pyoracle.abi.config_shape(cfg)
    rows = tr.core_rows[tr.head][list(picks)].cpu().numpy()
    owner = tr.core_owner[tr.head][list(picks)].cpu().numpy()
    for i, e in enumerate(picks):
        env = pyoracle.OracleEnv(cfg, seed + e)
        for f in range(frames):
            a = acts[f]
            price = a["price"][i].reshape(N, L) if "price" in a else None
            env.step(a["acc"][i].reshape(N, C), a["off"][i].reshape(N, L), price)
        o = env.observe()["acceptor"]   # [N, C, D]
        D = s["acc_obs_dim"]
        for c in range(C):
            ow = int(owner[i, c])
            if ow > 0:
                assert np.array_equal(rows[i, c, :D], o[ow - 1, c]), (e, c)
            for a_ in range(N):
                if a_ + 1 != ow:
                    assert o[a_, c, 0] == 0 and o[a_, c, 1] == -1, (e, c, a_)
