"""DQN units (§8(f) row 4, DQN env path): ms_dqn_act / ms_dqn_grad + HIP Adam against the torch-fp32
restatement of DQNmodules.py (oracle/dqn_ref.py), and the batched DQN loop on the env kernel."""
import importlib

import numpy as np
import pytest
import torch

from oracle.dqn_ref import RefDQNEntity, optimize_model_reference

pytestmark = pytest.mark.gpu


def _dqn(ms):
    return importlib.import_module("marl-scheduling_amd.dqn")


def _nets(dqn, G, D, A, seed):
    torch.manual_seed(seed)
    return [dqn.reference_qnet_params(D, A) for _ in range(G)]


@pytest.mark.parametrize("G,upg,D,stride,A", [(4, 1, 11, 12, 5), (6, 1, 6, 8, 3), (2, 3, 51, 52, 25), (1, 4, 195, 196, 97)])
def test_dqn_act_matches_reference(ms, G, upg, D, stride, A):
    dqn = _dqn(ms)
    nets = _nets(dqn, G, D, A, 0)
    q = dqn.GroupedQNet(nets, D, A).cuda()
    E, U = 301, G * upg
    gen = torch.Generator().manual_seed(1)
    obs = torch.zeros((E, U, stride), dtype=torch.int8)
    obs[..., :D] = torch.randint(-5, 13, (E, U, D), generator=gen, dtype=torch.int8)
    uni = torch.rand((2, E, U), generator=gen, dtype=torch.float64)
    eps = 0.4
    act, greedy = q.act(obs.cuda(), upg, eps, uniforms=uni.cuda())
    act, greedy = act.cpu().long(), greedy.cpu().long()
    for g in range(G):
        ref = RefDQNEntity(*[n[k] for n in nets[g:g + 1] for k in ("w1", "b1", "w2", "b2")])
        units = list(range(g * upg, (g + 1) * upg))
        with torch.no_grad():
            qv = ref(obs[:, units, :D].reshape(-1, D).long()).reshape(E, upg, A)
        top2 = qv.topk(2, dim=-1).values
        clear = (top2[..., 0] - top2[..., 1]) > 1e-5 * (1 + top2[..., 0].abs())
        want = qv.argmax(-1)
        got = greedy[:, units]
        assert torch.equal(got[clear], want[clear])
        explore = ~(uni[0][:, units] > eps)
        rnd = (uni[1][:, units] * A).long().clamp(max=A - 1)
        assert torch.equal(act[:, units][explore], rnd[explore])
        assert torch.equal(act[:, units][~explore], got[~explore])


@pytest.mark.parametrize("G,upg,D,stride,A,E,cap,B", [(4, 1, 11, 12, 5, 7, 30, 10), (3, 1, 6, 8, 3, 64, 50, 10),
                                                    (2, 2, 51, 52, 25, 33, 40, 10)])
@pytest.mark.parametrize("clip", [True, False])
def test_dqn_grad_and_adam_match_reference(ms, G, upg, D, stride, A, E, cap, B, clip):
    dqn = _dqn(ms)
    nets = _nets(dqn, G, D, A, 2)
    tnets = _nets(dqn, G, D, A, 3)
    hp = dqn.DQNHyper(grad_clip=1.0 if clip else 0.0)
    grp = dqn.DQNGroup(nets, D, A, 0.84, hp, "cuda")
    with torch.no_grad():
        for k in dqn.KEYS:
            getattr(grp.target, k).copy_(torch.stack([n[k] for n in tnets]).cuda())
    U = G * upg
    mem = dqn.ReplayMemories(E, U, cap, stride, "cuda")
    gen = torch.Generator().manual_seed(4)
    st = torch.zeros((E, U, cap, stride), dtype=torch.int8)
    st[..., :D] = torch.randint(-5, 13, (E, U, cap, D), generator=gen, dtype=torch.int8)
    nx = torch.zeros_like(st)
    nx[..., :D] = torch.randint(-5, 13, (E, U, cap, D), generator=gen, dtype=torch.int8)
    acts = torch.randint(0, A, (E, U, cap), generator=gen, dtype=torch.int8)
    rew = torch.randint(-20, 21, (E, U, cap), generator=gen).float()
    mem.states.copy_(st)
    mem.next_states.copy_(nx)
    mem.actions.copy_(acts)
    mem.rewards.copy_(rew)
    samples = torch.randint(0, cap, (E, U, B), generator=gen, dtype=torch.int32)
    loss = grp.optimize(mem, samples.cuda(), units_per_group=upg).cpu()
    for g in range(G):
        pol = RefDQNEntity(*[nets[g][k] for k in dqn.KEYS])
        tgt = RefDQNEntity(*[tnets[g][k] for k in dqn.KEYS])
        opt = torch.optim.Adam(pol.parameters())
        units = list(range(g * upg, (g + 1) * upg))
        idx = samples[:, units].long()                                   # [E, upg, B]
        ei = torch.arange(E)[:, None, None].expand_as(idx)
        ui = torch.tensor(units)[None, :, None].expand_as(idx)
        s = st[ei, ui, idx][..., :D].reshape(-1, D).long()
        s1 = nx[ei, ui, idx][..., :D].reshape(-1, D).long()
        a = acts[ei, ui, idx].reshape(-1)
        r = rew[ei, ui, idx].reshape(-1).long()
        want_loss = optimize_model_reference(pol, tgt, opt, s, a, s1, r, 0.84, clip=clip)
        assert abs(float(loss[g]) - float(want_loss)) <= 1e-5 * max(1.0, abs(float(want_loss))), (g, loss[g], want_loss)
        for k, p in zip(dqn.KEYS, pol.params()):
            got_g = getattr(grp.policy, k).grad[g].cpu()
            scale = p.grad.abs().max().item() + 1e-12
            assert (got_g - p.grad).abs().max().item() <= 1e-4 * scale + 1e-7, k
            got_w = getattr(grp.policy, k)[g].detach().cpu()
            np.testing.assert_allclose(got_w.numpy(), p.detach().numpy(), rtol=1e-4, atol=1e-6)


def test_replay_memory_push_semantics(ms):
    """ReplayMemory.push (DQNmodules.py:19-25): sequential slots, then the slot-(capacity-1) edge where one
    push fills nextFreeIndex and also overwrites a random index, then random replacement only."""
    dqn = _dqn(ms)
    E, U, cap, stride = 2, 3, 4, 4
    mem = dqn.ReplayMemories(E, U, cap, stride, "cuda")
    draws = []

    def repl():
        i = torch.full((E, U), len(draws) % cap, dtype=torch.long, device="cuda")
        draws.append(i)
        return i

    for t in range(6):
        s = torch.full((E, U, stride), t, dtype=torch.int8, device="cuda")
        mem.push(s, s[..., 0], s[..., 0].float(), s + 1, repl)
    # pushes 0, 1, 2 fill slots 0..2; push 2 reaches nextFreeIndex 3 == cap - 1 and also replaces slot 0;
    # pushes 3..5 replace slots 1, 2, 3 (the draw counter) only
    assert mem.next_free == cap - 1 and len(draws) == 4
    got = mem.actions[0, 0].cpu().tolist()
    assert got == [2, 3, 4, 5]


@pytest.mark.parametrize("name", ["cfg1", "cfg2"])
def test_dqn_trainer_runs_episodes(ms, name):
    dqn = _dqn(ms)
    cfg = ms.abi.named_config(name)
    hp = dqn.DQNHyper(replay_memory_size=64)
    tr = dqn.DQNTrainer(cfg, n_envs=128, hyper=hp, seed=1, episode_length=20)
    w0 = tr.acc.policy.w1.detach().clone()
    for _ in range(3):
        tr.episode()
    assert tr.flags() == 0 and tr.round == 60
    assert tr.mem_acc.next_free == 57
    assert torch.isfinite(tr.last_losses["acc"]).all() and torch.isfinite(tr.last_losses["off"]).all()
    assert not torch.equal(w0, tr.acc.policy.w1.detach())
    # the target nets were synced after episodes 0 and 2
    assert torch.equal(tr.acc.target.w1, tr.acc.policy.w1.detach())
