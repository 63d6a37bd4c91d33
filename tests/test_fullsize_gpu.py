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

* Every (draw, epoch) step of both PPO trainers re-synced (cfg3: all three unit types, agents 0 and 5;
  cfg4: one acceptor, one offer and one price unit): before each step the reference takes the HIP
  path's current weights and Adam state, so each step's own loss is held to the north star's 1e-5
  relative, its gradient to 1e-4 of the tensor's scale, and the HIP Adam's new weights to torch's
  Adam formula applied to the HIP gradient.

Returns are per replica (E = 1 semantics of PPOmodules.py:548-560), rows r = t * E + e.
Tolerances of the whole-update comparisons (no re-sync): the first draw's loss 1e-5 relative; after
an Adam step the weights agree within 1e-4 relative (Adam divides by sqrt(v), which amplifies last-ulp
gradient order differences), so later draws' losses there are held to 1e-4."""
import importlib
import random

import numpy as np
import pytest
import torch

from oracle import pyoracle
from oracle.ppo_ref import RefPPO, grad_abs_bound
from tests.replay import oracle_replay as _oracle_replay

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


def _cfg4_run(seed):
    tr = _tr().Trainer.from_named("cfg4", n_envs=8192, seed=seed, device="cuda:0")
    assert tr.arch == "divided" and tr.E == 8192 and tr.N == 16 and tr.C == 16
    return tr


def _resync_ref(tr, u, g):
    """A one-epoch RefPPO in float64 holding group g's current weights and HipAdam state (exp_avg,
    exp_avg_sq, step): its loss and gradient carry no rounding error of their own at this scale."""
    hp = tr.hp
    ref = RefPPO(u.D, u.group.policy.A, hp.lr_actor, hp.lr_critic, u.group.gamma, hp.eps_clip, 1)
    ref.policy.double()
    flat = ref.policy.flat()
    with torch.no_grad():
        for k, v in flat.items():
            v.copy_(getattr(u.group.policy, k)[g].detach().cpu().double())
    ref.policy.cuda()
    opt = u.group.hip_optimizer
    for k, v in flat.items():
        st = opt.state[getattr(u.group.policy, k)]
        ref.optimizer.state[v] = dict(step=torch.tensor(float(opt.step_count)), exp_avg=st["exp_avg"][g].double(),
                                      exp_avg_sq=st["exp_avg_sq"][g].double())
    return ref


# The gradient's per-element error bar. ms_ppo_grad sums R = T * E per-row terms in f32:
# per-row terms carry the f32 forward / backward's relative error (a few 2^-24, the fast exp / tanh / log ~2^-22),
# and the tile partials, the blocks' partials (k_ppo_reduce, fixed order) and the common rows' virtual tile add
# ~log2(R) = 21 (cfg3 / cfg4) rounding steps of 2^-24 on a running sum bounded by the terms' magnitudes, so
# |error| <= (21 + ~16) * 2^-24 * sum_r |term_r| ~ 2.2e-6 * sum_r |term_r| per element. Bar: 1e-5 of the terms'
# sum (4x margin). A tensor whose rows cancel (cfg4 acceptor 37's w3: its largest element 2.2e-4 against terms
# summing far higher) shows a large error against its own scale within this bar. The common rows' int64 sums
# (2^-28 per row, k_ppo_grad kCommonRow / k_own_scan) add at most R_common * 2^-29 / R <= 2^-29 to a logit's
# derivative: _GRAD_FLOOR covers it with the downstream factors (|h2| <= 1, |W| * |x| <= ~10).
_GRAD_REL = 1e-5
_GRAD_FLOOR = 2e-8


def _assert_resynced(report):
    """The per-step bars of _resynced_update over every recorded step."""
    for st in report:
        tag = st["tag"]
        np.testing.assert_allclose(st["loss"], st["want"], rtol=1e-5, atol=1e-6, err_msg=tag)
        for k, (e, sc, rb, bmax) in st["grad"].items():
            # |error| <= _GRAD_REL * sum_rows |term| + _GRAD_FLOOR per element (derivation: _GRAD_REL)
            assert rb <= _GRAD_REL, (tag, k, e, sc, rb, bmax)
        for k, v in st["adam"].items():
            assert v[0] <= 1e-6 * max(abs(v[1]), 1e-3), (tag, k) + v
        for k, (frac, dmax, lr) in st["delta"].items():
            assert frac <= 0.01 and dmax <= 2 * lr + 1e-7, (tag, k, frac, dmax)


def _adam_replay(tr, k, w0, grad, m0, v0, step):
    """torch.optim.Adam's step (PPOmodules.py:100-105 param groups) of one tensor from (w0, m0, v0, step)
    with the given gradient: the weights the HIP Adam must produce from the HIP gradient."""
    p = torch.nn.Parameter(w0.clone())
    p.grad = grad.clone()
    lr = tr.hp.lr_critic if k.startswith("c") else tr.hp.lr_actor
    opt = torch.optim.Adam([p], lr=lr, foreach=False)
    opt.state[p] = dict(step=torch.tensor(float(step)), exp_avg=m0.clone(), exp_avg_sq=v0.clone())
    opt.step()
    return p.detach()


def _resynced_update(tr, picks, report):
    """The trainer's fused update run step by step: the closures Trainer._epochs builds (the kernels the
    update graph replays) and the HIP Adam. Before every (draw, epoch) step, group g of picks[name]
    is re-synced into a RefPPO that takes the same step on the same rows (PPOmodules.py:144-168,
    548-597): the step's loss within 1e-5 relative, its gradient within 1e-4 of each tensor's scale,
    the HIP Adam's weights == torch's Adam formula on the HIP gradient (1e-6 relative), and the
    weight delta against the reference's (1e-4 relative + 1e-4 lr absolute for at least 99 % of
    the elements; the rest are near-cancelled gradients whose Adam step sign is noise, none beyond
    2 lr)."""
    ppo = _ppo()
    keys = ppo.ACTOR_KEYS + ppo.CRITIC_KEYS
    T = tr.T
    sel = tr._draws()
    all_sel = {k: torch.cat(v).to(torch.int32) for k, v in sel.items()}
    counts = {k: [x.numel() for x in v] for k, v in sel.items()}
    for u in tr.units():
        seq = tr._epochs(u, all_sel[u.name], counts[u.name])
        K = u.group.K
        opt = u.group.hip_optimizer
        pol = u.group.policy
        for s, ep in enumerate(seq):
            d = s // K
            step0 = opt.step_count
            before = {g: {k: (getattr(pol, k)[g].detach().clone(), opt.state[getattr(pol, k)]["exp_avg"][g].clone(),
                              opt.state[getattr(pol, k)]["exp_avg_sq"][g].clone()) for k in keys}
                      for g in picks[u.name]}
            refs = {g: _resync_ref(tr, u, g) for g in picks[u.name]}
            rows = {g: _unit_rows(tr, u, int(sel[u.name][d][g]), T) for g in picks[u.name]}
            bounds = {g: grad_abs_bound(_resync_ref(tr, u, g).policy, rows[g][0].double(), rows[g][1],
                                        rows[g][2].double(), _returns(rows[g][3], u.group.gamma).cuda().double(),
                                        tr.hp.eps_clip) for g in picks[u.name]}
            loss = ep().cpu()
            grads = {g: {k: getattr(pol, k).grad[g].detach().clone() for k in keys} for g in picks[u.name]}
            opt.step()
            torch.cuda.synchronize()
            for g in picks[u.name]:
                x, act, lp, rw = rows[g]
                want, rgrad = refs[g].epoch(x.double(), act, lp.double(), _returns(rw, u.group.gamma).cuda().double())
                tag = "%s group %d step %d" % (u.name, g, s)
                rel = abs(float(loss[g]) - want) / max(abs(want), 1e-30)
                st = dict(tag=tag, loss=float(loss[g]), want=want, rel=rel, grad={}, adam={}, delta={})
                bound = bounds[g]
                for k in keys:
                    w0, m0, v0 = before[g][k]
                    sc = rgrad[k].abs().max().item()
                    err = (grads[g][k].double() - rgrad[k]).abs()
                    e = err.max().item()
                    # the error of each element against its rows' summed magnitudes (oracle grad_abs_bound)
                    rb = (err / (bound[k] + _GRAD_FLOOR / _GRAD_REL)).max().item()
                    st["grad"][k] = (e, sc, rb, bound[k].max().item())
                    w1 = getattr(pol, k)[g].detach()
                    want_w = _adam_replay(tr, k, w0, grads[g][k], m0, v0, step0)
                    da = (w1 - want_w).abs()
                    i = int(da.argmax())
                    st["adam"][k] = (da.max().item(), float(w0.flatten()[i]), float(w1.flatten()[i]),
                                     float(want_w.flatten()[i]), float(grads[g][k].flatten()[i]),
                                     float(m0.flatten()[i]), float(v0.flatten()[i]), step0)
                    lr = tr.hp.lr_critic if k.startswith("c") else tr.hp.lr_actor
                    dg, dr = (w1 - w0).double(), refs[g].policy.flat()[k].detach() - w0.double()
                    dd = (dg - dr).abs()
                    loose = dd > 1e-4 * dr.abs() + 1e-4 * lr
                    st["delta"][k] = (loose.float().mean().item(), dd.max().item(), lr)
                report.append(st)
                print("%s: loss %.7g want %.7g rel %.2e | grad err/scale %s | adam max %s | delta loose %s" % (
                    tag, st["loss"], want, rel,
                    " ".join("%s %.1e/%.1e (%.1e of terms)" % (k, v[0], v[1], v[2]) for k, v in st["grad"].items()),
                    " ".join("%s %.1e" % (k, v[0]) for k, v in st["adam"].items()),
                    " ".join("%s %.4f/%.1e" % (k, v[0], v[1]) for k, v in st["delta"].items())), flush=True)
                worst = max(st["adam"].items(), key=lambda kv: kv[1][0])
                print("   worst adam %s: d %.3e w0 %.9g w1 %.9g want %.9g g %.3e m0 %.3e v0 %.3e step %d"
                      % ((worst[0],) + worst[1]), flush=True)
        u.group.last_losses = []
        u.group.sync_old()
    tr._carry_last_observation()


def test_cfg3_every_update_step_resynced(ms):
    tr = _tr().Trainer.from_named("cfg3", seed=9, device="cuda:0")
    tr.rollout()
    torch.cuda.synchronize()
    assert tr.flags() == 0
    report = []
    _resynced_update(tr, {u.name: (0, 5) for u in tr.units()}, report)
    _assert_resynced(report)
    assert len(report) == 2 * sum(tr.hp.centralisation_sample * u.group.K for u in tr.units())


def test_cfg4_every_update_step_resynced(ms):
    tr = _cfg4_run(13)
    tr.rollout()
    torch.cuda.synchronize()
    assert tr.flags() == 0
    report = []
    _resynced_update(tr, dict(acceptor=(37,), offer=(5,), price=(20,)), report)
    _assert_resynced(report)
    assert len(report) == sum(u.group.K for u in tr.units())


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
