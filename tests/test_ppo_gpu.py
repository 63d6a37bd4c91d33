"""PPO kernels on the device vs the torch-fp32 CPU restatement (oracle/ppo_ref.py)."""
import importlib

import numpy as np
import pytest
import torch

from oracle.ppo_ref import RefPPO, act_reference

pytestmark = pytest.mark.gpu


def _ppo(ms):
    return importlib.import_module("marl-scheduling_amd.ppo")


@pytest.mark.parametrize("G,per_group,D,stride,A", [(8, 8, 51, 52, 25), (24, 1, 18, 20, 9), (1, 16, 27, 28, 13),
                                                     (8, 3, 4, 4, 13), (2, 5, 195, 196, 97), (3, 2, 11, 12, 5)])
def test_act_kernel_matches_reference(ms, G, per_group, D, stride, A):
    ppo = _ppo(ms)
    torch.manual_seed(0)
    net = ppo.GroupedActorCritic(G, D, A)
    E, U = 333, G * per_group
    gen = torch.Generator().manual_seed(1)
    obs = torch.zeros((E, U, stride), dtype=torch.int8)
    obs[..., :D] = torch.randint(-5, 13, (E, U, D), generator=gen, dtype=torch.int8)
    u = torch.rand((E, U), generator=gen)
    dnet = net.cuda()
    act, lp = dnet.act(obs.cuda(), U, seed=0, offset=0, uniforms=u.cuda())
    act, lp = act.cpu().long(), lp.cpu()
    for g in range(G):
        flat = {k: getattr(net, k)[g].detach().cpu() for k in ppo.ACTOR_KEYS}
        rows = obs[:, g * per_group:(g + 1) * per_group, :D].float()
        ra, rlp, probs = act_reference(flat, rows, u[:, g * per_group:(g + 1) * per_group])
        ga = act[:, g * per_group:(g + 1) * per_group]
        glp = lp[:, g * per_group:(g + 1) * per_group]
        mism = ga != ra
        if mism.any():  # only allowed when u sits on a CDF boundary (f32 rounding)
            cdf = torch.cumsum(probs, -1)
            uu = u[:, g * per_group:(g + 1) * per_group][mism]
            gap = (cdf[mism] - uu.unsqueeze(-1)).abs().min(-1).values
            assert (gap < 1e-5).all()
        same = ~mism
        np.testing.assert_allclose(glp[same].numpy(), rlp[same].numpy(), rtol=1e-5, atol=2e-6)


def _common_row(D, stride, O):
    return torch.tensor([0, -1, -1] + [-2] * (2 * O) + [0] * (stride - D), dtype=torch.int8)


@pytest.mark.parametrize("G,per_group,O,A,frac", [(8, 8, 24, 25, 0.85), (8, 8, 24, 25, 0.0), (8, 8, 24, 25, 1.0),
                                                  (1, 16, 12, 13, 0.5), (3, 2, 4, 5, 0.9), (2, 5, 96, 97, 0.8)])
@pytest.mark.parametrize("ext_u", [False, True])
def test_act_common_rows_bit_identical(ms, G, per_group, O, A, frac, ext_u):
    """ms_policy_act_common == ms_policy_act bit for bit (actions and log-probs) on acceptor-shaped
    observations where a fraction of the rows equal the common (not-owned-core) row, incl. rows
    that differ from it in one byte only."""
    ppo = _ppo(ms)
    D = 3 + 2 * O
    stride = (D + 3) // 4 * 4
    torch.manual_seed(5)
    net = ppo.GroupedActorCritic(G, D, A).cuda()
    E, U = 1001, G * per_group
    gen = torch.Generator().manual_seed(6)
    crow = _common_row(D, stride, O)
    obs = torch.zeros((E, U, stride), dtype=torch.int8)
    obs[..., :D] = torch.randint(-5, 13, (E, U, D), generator=gen, dtype=torch.int8)
    pick = torch.rand((E, U), generator=gen) < frac
    obs[pick] = crow
    near = (torch.rand((E, U), generator=gen) < 0.02) & pick  # one byte off the common row
    col = torch.randint(0, D, (E, U), generator=gen)
    obs[near, col[near]] = 7
    u = torch.rand((E, U), generator=gen).cuda() if ext_u else None
    dobs = obs.cuda()
    a0, l0 = net.act(dobs, U, seed=3, offset=11, uniforms=u)
    a1, l1 = net.act(dobs, U, seed=3, offset=11, uniforms=u, common_row=crow.cuda())
    assert torch.equal(a0, a1)
    assert torch.equal(l0.view(torch.int32), l1.view(torch.int32))
    # the same with ms_act_prepare's fragments (the common-row table made once, not per wave)
    frag = ppo.ActFrag(net, stride, crow.cuda())
    frag.build(net)
    a2, l2 = net.act(dobs, U, seed=3, offset=11, uniforms=u, common_row=crow.cuda(), frag=frag)
    a3, l3 = net.act(dobs, U, seed=3, offset=11, uniforms=u, frag=frag)
    for a, l in ((a2, l2), (a3, l3)):
        assert torch.equal(a0, a)
        assert torch.equal(l0.view(torch.int32), l.view(torch.int32))


def test_act_kernel_sampling_distribution(ms):
    """Philox sampling follows the policy distribution (chi-square-like bound)."""
    ppo = _ppo(ms)
    torch.manual_seed(3)
    net = ppo.GroupedActorCritic(1, 6, 4).cuda()
    E = 200000
    obs = torch.zeros((E, 1, 8), dtype=torch.int8, device="cuda")
    obs[..., :6] = torch.tensor([1, 2, -1, 3, 0, 5], dtype=torch.int8)
    act, lp = net.act(obs, 1, seed=9, offset=4)
    counts = torch.bincount(act.long().flatten(), minlength=4).cpu().double()
    probs = torch.exp(lp.cpu().double().flatten())
    p = torch.zeros(4, dtype=torch.double)
    for a in range(4):
        sel = act.cpu().flatten() == a
        if sel.any():
            p[a] = probs[sel][0]
    expected = p * E
    assert ((counts - expected).abs() <= 5 * expected.sqrt() + 5).all(), (counts, expected)
    # different offsets give different draws, same offset reproduces
    a2, _ = net.act(obs, 1, seed=9, offset=4)
    a3, _ = net.act(obs, 1, seed=9, offset=5)
    assert torch.equal(act, a2) and not torch.equal(act, a3)


def test_returns_kernel_matches_reference(ms):
    ppo = _ppo(ms)
    gen = torch.Generator().manual_seed(2)
    T, M = 200, 37
    r = torch.randint(-20, 30, (T, M), generator=gen).float()
    r[:, 3] = 0.5 * torch.randint(-4, 4, (T,), generator=gen).float()
    ref = RefPPO(4, 3, 0.1, 0.1, 0.8733, 0.2, 1)
    got = ppo.discounted_returns(r.cuda(), 0.8733).cpu()
    for m in range(M):
        want = ref.returns([float(x) for x in r[:, m]])
        np.testing.assert_allclose(got[m].numpy(), want.numpy(), rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("T", [60, 200])  # 200: the kernel holding each sequence in registers
@pytest.mark.parametrize("dtype", [torch.int32, torch.float32])
def test_unit_returns_gathers_and_matches_reference(ms, dtype, T):
    ppo = _ppo(ms)
    gen = torch.Generator().manual_seed(8)
    E, U, G = 33, 24, 8
    r = torch.randint(-20, 30, (T, E, U), generator=gen)
    r = r.to(dtype) if dtype == torch.int32 else (0.5 * r).float()
    sel = torch.randint(0, U, (G,), generator=gen).to(torch.int32)
    ref = RefPPO(4, 3, 0.1, 0.1, 0.9, 0.2, 1)
    got = ppo.unit_returns(r.cuda(), sel.cuda(), 0.9).cpu()
    assert got.shape == (T, E, G)
    for e in (0, 7, E - 1):
        for g in range(G):
            want = ref.returns([float(x) for x in r[:, e, sel[g]]])
            np.testing.assert_allclose(got[:, e, g].numpy(), want.numpy(), rtol=1e-5, atol=2e-6)


def test_grouped_update_on_device_matches_reference(ms):
    ppo = _ppo(ms)
    G, T, D, A, K = 4, 200, 51, 25, 2
    torch.manual_seed(11)
    refs = [RefPPO(D, A, 0.003, 0.01, 0.95, 0.2, K) for _ in range(G)]
    torch.manual_seed(11)
    grp = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.95, 0.2, K, device="cuda")
    gen = torch.Generator().manual_seed(4)
    states = torch.randint(-5, 13, (G, T, D), generator=gen).float()
    actions = torch.randint(0, A, (G, T), generator=gen)
    old_lp = -torch.rand((G, T), generator=gen) * 3
    rewards = torch.randint(-6, 13, (G, T), generator=gen).float()
    rets = torch.stack([refs[g].returns(rewards[g].tolist()) for g in range(G)])
    ref_losses = np.array([refs[g].update(states[g], actions[g], old_lp[g], rets[g]) for g in range(G)])
    dev_rets = ppo.discounted_returns(rewards.T.contiguous().cuda(), 0.95)
    np.testing.assert_allclose(dev_rets.cpu().numpy(), rets.numpy(), rtol=1e-5, atol=2e-6)
    losses = grp.update(states.cuda(), actions.cuda(), old_lp.cuda(), dev_rets)
    np.testing.assert_allclose(torch.stack(losses).T.cpu().numpy(), ref_losses, rtol=1e-5, atol=1e-5)
    for g in range(G):
        for k, v in refs[g].policy.flat().items():
            np.testing.assert_allclose(getattr(grp.policy, k)[g].detach().cpu().numpy(), v.detach().numpy(),
                                       rtol=1e-4, atol=1e-5, err_msg=k)


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3"])
def test_trainer_iterations(ms, name):
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    tr = tr_mod.Trainer.from_named(name, n_envs=64, update_step=50, seed=3, device="cuda:0")
    for _ in range(2):
        losses = tr.iteration()
        for k, v in losses.items():
            assert torch.isfinite(v).all(), k
    assert tr.flags() == 0
    assert tr.env.round == 100


def _rand_batch(G, T, E, U, D, stride, A, seed):
    gen = torch.Generator().manual_seed(seed)
    R = T * E
    states = torch.zeros((R, U, stride), dtype=torch.int8)
    states[..., :D] = torch.randint(-5, 13, (R, U, D), generator=gen, dtype=torch.int8)
    actions = torch.randint(0, A, (R, U), generator=gen).to(torch.int8)
    old_lp = -torch.rand((R, U), generator=gen) * 3
    ret = torch.randn((E, G, T), generator=gen)
    return states, actions, old_lp, ret


@pytest.mark.parametrize("G,T,E,U,D,stride,A,K", [(8, 20, 37, 64, 51, 52, 25, 1), (8, 13, 11, 24, 18, 20, 9, 2),
                                                   (8, 9, 50, 24, 4, 4, 13, 1), (3, 7, 9, 3, 11, 12, 5, 2),
                                                   (2, 5, 16, 4, 195, 196, 97, 1), (2, 6, 21, 3, 16, 16, 5, 1),
                                                   (1, 3, 333, 2, 99, 100, 49, 1), (4, 8, 40, 6, 34, 36, 17, 2)])
def test_fused_grad_matches_autograd(ms, G, T, E, U, D, stride, A, K):
    """A = 17 / 49 with 16 < D + 1 <= 64 / 64 < D + 1 <= 128: the single-action last tile (kX1)."""
    ppo = _ppo(ms)
    torch.manual_seed(21)
    ref = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.9, 0.2, K, device="cuda")
    torch.manual_seed(21)
    fus = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.9, 0.2, K, device="cuda")
    states, actions, old_lp, ret = _rand_batch(G, T, E, U, D, stride, A, 5)
    u_sel = torch.randint(0, U, (G,), generator=torch.Generator().manual_seed(1))
    R = T * E
    # torch reference batch: rows r = t*E + e of unit u_sel[g]
    x = states[:, u_sel, :D].permute(1, 0, 2).float().cuda()
    a = actions[:, u_sel].T.long().cuda()
    lp = old_lp[:, u_sel].T.contiguous().cuda()
    rt = ret.permute(1, 2, 0).reshape(G, R).cuda()  # [G][t][e] -> r = t*E + e
    ref_losses = ref.update(x, a, lp, rt)
    ref_grads = {k: getattr(ref.policy, k).grad.clone() for k in ppo.ACTOR_KEYS + ppo.CRITIC_KEYS}
    fus_losses = fus.update_fused(states.cuda(), actions.cuda(), old_lp.cuda(), ret.permute(2, 0, 1).contiguous().cuda(),
                                  u_sel.to(torch.int32).cuda(), T, E)
    for rl, fl in zip(ref_losses, fus_losses):
        np.testing.assert_allclose(fl.cpu().numpy(), rl.cpu().numpy(), rtol=1e-5, atol=1e-6)
    for k, g in ref_grads.items():
        fg = getattr(fus.policy, k).grad
        scale = g.abs().max().item() + 1e-12
        err = (fg - g).abs().max().item()
        assert err <= 1e-4 * scale + 1e-7, (k, err, scale)
    # after Adam: Adam's first steps move every weight by about lr * sign(g), so elements whose
    # gradient is at the f32 noise floor (|g| < 1e-3 max|g|) may move either way; all others agree
    for k in ppo.ACTOR_KEYS + ppo.CRITIC_KEYS:
        wf = getattr(fus.policy, k).detach().cpu()
        wr = getattr(ref.policy, k).detach().cpu()
        g = ref_grads[k].abs().cpu()
        firm = g > 1e-3 * g.max()
        np.testing.assert_allclose(wf[firm].numpy(), wr[firm].numpy(), rtol=1e-4, atol=1e-5, err_msg=k)
        lr = 0.003 if k in ppo.ACTOR_KEYS else 0.01
        assert ((wf - wr)[~firm].abs() <= 2 * lr * K + 1e-6).all(), k


@pytest.mark.parametrize("G,T,E,U,O,A,K,frac", [(8, 20, 37, 64, 24, 25, 1, 0.9), (8, 13, 111, 8, 24, 25, 2, 1.0),
                                                  (3, 7, 90, 3, 4, 5, 2, 0.5), (2, 6, 301, 4, 12, 13, 1, 0.0),
                                                  (1, 41, 250, 2, 48, 49, 1, 0.95)])
def test_fused_grad_common_rows_matches_autograd(ms, G, T, E, U, O, A, K, frac):
    """ms_ppo_grad with common_row (rows equal to it share one forward and one summed backward)
    against torch autograd of PPO.update on the same rows; chunks of > 1024 rows per wave exercise
    the segment carry-over of the listed rows."""
    ppo = _ppo(ms)
    D = 3 + 2 * O
    stride = (D + 3) // 4 * 4
    torch.manual_seed(22)
    ref = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.9, 0.2, K, device="cuda")
    torch.manual_seed(22)
    fus = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.9, 0.2, K, device="cuda")
    states, actions, old_lp, ret = _rand_batch(G, T, E, U, D, stride, A, 6)
    crow = _common_row(D, stride, O)
    gen = torch.Generator().manual_seed(7)
    pick = torch.rand(states.shape[:2], generator=gen) < frac
    states[pick] = crow
    u_sel = torch.randint(0, U, (G,), generator=torch.Generator().manual_seed(2))
    R = T * E
    x = states[:, u_sel, :D].permute(1, 0, 2).float().cuda()
    a = actions[:, u_sel].T.long().cuda()
    lp = old_lp[:, u_sel].T.contiguous().cuda()
    rt = ret.permute(1, 2, 0).reshape(G, R).cuda()
    ref_losses = ref.update(x, a, lp, rt)
    ref_grads = {k: getattr(ref.policy, k).grad.clone() for k in ppo.ACTOR_KEYS + ppo.CRITIC_KEYS}
    fus_losses = fus.update_fused(states.cuda(), actions.cuda(), old_lp.cuda(), ret.permute(2, 0, 1).contiguous().cuda(),
                                  u_sel.to(torch.int32).cuda(), T, E, common_row=crow.cuda())
    for rl, fl in zip(ref_losses, fus_losses):
        np.testing.assert_allclose(fl.cpu().numpy(), rl.cpu().numpy(), rtol=1e-5, atol=1e-6)
    for k, g in ref_grads.items():
        fg = getattr(fus.policy, k).grad
        scale = g.abs().max().item() + 1e-12
        err = (fg - g).abs().max().item()
        assert err <= 1e-4 * scale + 1e-7, (k, err, scale)


@pytest.mark.parametrize("G,T,E,U,A,K,n_keys", [(8, 20, 300, 24, 16, 2, 40), (4, 13, 700, 6, 13, 1, 3000),
                                                 (2, 50, 2000, 3, 9, 1, 0), (2, 9, 400, 3, 20, 1, -1)])
def test_fused_grad_keyed_rows_matches_autograd(ms, G, T, E, U, A, K, n_keys):
    """ms_ppo_grad on 4-byte rows (the price chooser's input, PPOmodules.py:327-330): each group's
    distinct rows get one forward and one backward, every row adds its loss derivatives to its
    distinct row's fixed-point sums. n_keys distinct rows per batch (3000: more than one scan pass
    of ranks; 0: bytes uniform in [-8, 24), more distinct rows than ranks, and -1: bytes over the
    whole int8 range, outside the dense index: both send the groups to the tile path);
    checked against torch autograd and against the same kernel with keying off (row_keys = -1),
    and twice in a row for bit-identical gradients."""
    ppo = _ppo(ms)
    D, stride = 4, 4
    gen = torch.Generator().manual_seed(8)
    R = T * E
    if n_keys > 0:
        pool = torch.randint(-5, 13, (n_keys, 4), generator=gen, dtype=torch.int8)
        pool[0] = -5  # the price chooser's [-5, -5, -5, -5] row (no offer), a tenth of all rows
        idx = torch.randint(0, n_keys, (R, U), generator=gen)
        idx[torch.rand((R, U), generator=gen) < 0.1] = 0
        states = pool[idx]
    elif n_keys == 0:
        states = torch.randint(-8, 24, (R, U, 4), generator=gen, dtype=torch.int8)
    else:
        states = torch.randint(-128, 127, (R, U, 4), generator=gen, dtype=torch.int8)
    actions = torch.randint(0, A, (R, U), generator=gen).to(torch.int8)
    old_lp = -torch.rand((R, U), generator=gen) * 3
    ret = torch.randn((E, G, T), generator=gen)
    u_sel = torch.randint(0, U, (G,), generator=torch.Generator().manual_seed(3))
    x = states[:, u_sel, :D].permute(1, 0, 2).float().cuda()
    a = actions[:, u_sel].T.long().cuda()
    lp = old_lp[:, u_sel].T.contiguous().cuda()
    rt = ret.permute(1, 2, 0).reshape(G, R).cuda()
    torch.manual_seed(23)
    ref = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.9, 0.2, K, device="cuda")
    ref_losses = ref.update(x, a, lp, rt)
    ref_grads = {k: getattr(ref.policy, k).grad.clone() for k in ppo.ACTOR_KEYS + ppo.CRITIC_KEYS}
    args = (states.cuda(), actions.cuda(), old_lp.cuda(), ret.permute(2, 0, 1).contiguous().cuda(),
            u_sel.to(torch.int32).cuda(), T, E)
    runs = []
    for keys in (0, 0, -1):
        torch.manual_seed(23)
        fus = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.9, 0.2, K, device="cuda")
        fus.row_keys = keys
        losses = fus.update_fused(*args)
        runs.append((losses, {k: getattr(fus.policy, k).grad.clone() for k in ref_grads}))
    for losses, grads in runs:
        for rl, fl in zip(ref_losses, losses):
            np.testing.assert_allclose(fl.cpu().numpy(), rl.cpu().numpy(), rtol=1e-5, atol=1e-6)
        for k, g in ref_grads.items():
            scale = g.abs().max().item() + 1e-12
            err = (grads[k] - g).abs().max().item()
            assert err <= 1e-4 * scale + 1e-7, (k, err, scale)
    for k in ref_grads:  # integer sums: the keyed gradient does not depend on the atomics' order
        assert torch.equal(runs[0][1][k], runs[1][1][k]), k
    # unit-major rollout rows ([U][R], the trainer's price chooser rings): the same gradients bit for bit,
    # keyed and on the tile path
    um = (states.permute(1, 0, 2).contiguous().cuda(), actions.T.contiguous().cuda(), old_lp.T.contiguous().cuda())
    for keys, base in ((0, runs[0]), (-1, runs[2])):
        torch.manual_seed(23)
        fus = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.9, 0.2, K, device="cuda")
        fus.row_keys = keys
        losses = fus.update_fused(*um, *args[3:], unit_major=True)
        for rl, fl in zip(base[0], losses):
            assert torch.equal(rl, fl), keys
        for k in ref_grads:
            assert torch.equal(getattr(fus.policy, k).grad, base[1][k]), (keys, k)


@pytest.mark.parametrize("G,per_group,N,C,O,E", [(8, 8, 8, 8, 24, 1001), (1, 16, 4, 4, 12, 333),
                                                 (32, 32, 32, 32, 96, 65), (3, 4, 3, 4, 9, 200)])
@pytest.mark.parametrize("ext_u", [False, True])
def test_act_compact_bit_identical(ms, G, per_group, N, C, O, E, ext_u):
    """ms_policy_act_compact on (core rows, owners) == ms_policy_act_common on the [E][N*C] rows they
    regenerate (Agent.py:167-212), bit for bit; owners include the auctioneer (0)."""
    ppo = _ppo(ms)
    D, A = 3 + 2 * O, O + 1
    stride = (D + 3) // 4 * 4
    U = N * C
    assert U == G * per_group
    torch.manual_seed(7)
    net = ppo.GroupedActorCritic(G, D, A).cuda()
    gen = torch.Generator().manual_seed(8)
    rows = torch.zeros((E, C, stride), dtype=torch.int8)
    rows[..., :D] = torch.randint(-5, 13, (E, C, D), generator=gen, dtype=torch.int8)
    owner = torch.randint(0, N + 1, (E, C), generator=gen, dtype=torch.int8)
    crow = _common_row(D, stride, O).cuda()
    rows, owner = rows.cuda(), owner.cuda()
    full = ppo.regen_acceptor_rows(rows, owner, crow, N).contiguous()
    assert full.shape == (E, U, stride)
    u = torch.rand((E, U), generator=gen).cuda() if ext_u else None
    a0, l0 = net.act(full, U, seed=3, offset=11, uniforms=u, common_row=crow)
    a1, l1 = net.act_compact(rows, owner, U, 3, 11, crow, uniforms=u)
    assert torch.equal(a0, a1)
    assert torch.equal(l0.view(torch.int32), l1.view(torch.int32))


@pytest.mark.parametrize("G,T,E,N,C,O,K", [(8, 20, 37, 8, 8, 24, 1), (2, 9, 301, 4, 4, 12, 2), (1, 41, 250, 2, 3, 6, 1)])
def test_fused_grad_compact_rows_bit_identical(ms, G, T, E, N, C, O, K):
    """ms_ppo_grad on compact acceptor rows (core rows + owners) == ms_ppo_grad with common_row on
    the regenerated [R][N*C] rows, bit for bit (same rows in the same order through the same
    arithmetic), and within tolerance of torch autograd."""
    ppo = _ppo(ms)
    D, A = 3 + 2 * O, O + 1
    stride = (D + 3) // 4 * 4
    R, U = T * E, N * C
    gen = torch.Generator().manual_seed(9)
    rows = torch.zeros((R, C, stride), dtype=torch.int8)
    rows[..., :D] = torch.randint(-5, 13, (R, C, D), generator=gen, dtype=torch.int8)
    owner = torch.randint(0, N + 1, (R, C), generator=gen, dtype=torch.int8)
    actions = torch.randint(0, A, (R, U), generator=gen).to(torch.int8)
    old_lp = -torch.rand((R, U), generator=gen) * 3
    ret = torch.randn((T, E, G), generator=gen)
    u_sel = torch.randint(0, U, (G,), generator=torch.Generator().manual_seed(4)).to(torch.int32)
    crow = _common_row(D, stride, O).cuda()
    rows, owner = rows.cuda(), owner.cuda()
    full = ppo.regen_acceptor_rows(rows, owner, crow, N).contiguous()
    args = (actions.cuda(), old_lp.cuda(), ret.cuda(), u_sel.cuda(), T, E)
    res = []
    for compact in (False, True):
        torch.manual_seed(24)
        grp = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.9, 0.2, K, device="cuda")
        if compact:
            losses = grp.update_fused(rows, *args, common_row=crow, core_owner=owner)
        else:
            losses = grp.update_fused(full, *args, common_row=crow)
        res.append((losses, {k: getattr(grp.policy, k).detach().clone() for k in ppo.ACTOR_KEYS + ppo.CRITIC_KEYS}))
    for l0, l1 in zip(res[0][0], res[1][0]):
        assert torch.equal(l0, l1)
    for k in res[0][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k


@pytest.mark.parametrize("N,C,G,T,E,K,shuffle", [(8, 8, 64, 6, 1700, 2, False), (10, 10, 70, 3, 2999, 1, True),
                                                  (16, 16, 256, 4, 1100, 1, False)])
def test_fused_grad_compact_many_groups_matches_autograd(ms, N, C, G, T, E, K, shuffle):
    """ms_ppo_grad on compact acceptor rows with >= 64 groups (the divided acceptors, cfg4: k_own_scan
    sums the common rows of 64 groups per pass, the tiles run the marked rows) against torch autograd
    of PPO.update on the regenerated rows (Agent.py:167-212), including a unit map that is not the
    identity, a group count that leaves a partial lane block, and R over several scan blocks with a
    partial last chunk; and twice in a row for bit-identical gradients."""
    ppo = _ppo(ms)
    O = 3 * N
    D, A = 3 + 2 * O, O + 1
    stride = (D + 3) // 4 * 4
    R, U = T * E, N * C
    gen = torch.Generator().manual_seed(31)
    rows = torch.zeros((R, C, stride), dtype=torch.int8)
    rows[..., :D] = torch.randint(-5, 13, (R, C, D), generator=gen, dtype=torch.int8)
    owner = torch.randint(0, N + 1, (R, C), generator=gen, dtype=torch.int8)
    actions = torch.randint(0, A, (R, U), generator=gen).to(torch.int8)
    old_lp = -torch.rand((R, U), generator=gen) * 3
    ret = torch.randn((T, E, G), generator=gen)
    u_sel = (torch.randperm(U, generator=gen)[:G] if shuffle else torch.arange(G)).to(torch.int32)
    crow = _common_row(D, stride, O).cuda()
    rows, owner = rows.cuda(), owner.cuda()
    full = ppo.regen_acceptor_rows(rows, owner, crow, N).contiguous()
    us = u_sel.long().cuda()
    x = full[:, us, :D].permute(1, 0, 2).float()
    a = actions.cuda()[:, us].T.long()
    lp = old_lp.cuda()[:, us].T.contiguous()
    rt = ret.cuda().permute(2, 0, 1).reshape(G, R)
    torch.manual_seed(25)
    ref = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.9, 0.2, K, device="cuda")
    ref_losses = ref.update(x, a, lp, rt)
    ref_grads = {k: getattr(ref.policy, k).grad.clone() for k in ppo.ACTOR_KEYS + ppo.CRITIC_KEYS}
    del x, full
    runs = []
    for _ in range(2):
        torch.manual_seed(25)
        fus = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.9, 0.2, K, device="cuda")
        losses = fus.update_fused(rows, actions.cuda(), old_lp.cuda(), ret.cuda(), u_sel.cuda(), T, E,
                                  common_row=crow, core_owner=owner)
        runs.append((losses, {k: getattr(fus.policy, k).grad.clone() for k in ref_grads}))
    for rl, fl in zip(ref_losses, runs[0][0]):
        np.testing.assert_allclose(fl.cpu().numpy(), rl.cpu().numpy(), rtol=1e-5, atol=1e-6)
    for k, g in ref_grads.items():  # (K = 2: the second epoch's gradient, after one Adam step each)
        fg = runs[0][1][k]
        scale = g.abs().max().item() + 1e-12
        err = (fg - g).abs().max().item()
        assert err <= (1e-4 if K == 1 else 1e-3) * scale + 1e-7, (k, err, scale)
    for k in ref_grads:
        assert torch.equal(runs[0][1][k], runs[1][1][k]), k


@pytest.mark.parametrize("N,C,L,O,E,G", [(4, 4, 3, 12, 4096, 1), (4, 4, 3, 12, 301, 1), (8, 8, 3, 24, 513, 8),
                                         (16, 16, 3, 48, 97, 1)])
def test_act_round_fixed_matches_separate_calls(ms, N, C, L, O, E, G):
    """ms_act_round_free with price_chooser NULL (a fixed-price round: the offer units' net and the compact
    acceptors in one launch, the paired kernel for cfg2's shapes, two launches otherwise) == ms_policy_act +
    ms_policy_act_compact, bit for bit, with and without act fragments, and with a replica base."""
    ppo = _ppo(ms)
    torch.manual_seed(13)
    D_off, A_off, D_acc, A_acc = 2 * C + 2, C + 1, 3 + 2 * O, O + 1
    s_off, s_acc = (D_off + 3) & ~3, (D_acc + 3) & ~3
    off = ppo.GroupedActorCritic(G, D_off, A_off).cuda()
    acc = ppo.GroupedActorCritic(G, D_acc, A_acc).cuda()
    gen = torch.Generator().manual_seed(14)
    off_obs = torch.zeros((E, N * L, s_off), dtype=torch.int8)
    off_obs[..., :D_off] = torch.randint(-1, 13, (E, N * L, D_off), generator=gen, dtype=torch.int8)
    rows = torch.zeros((E, C, s_acc), dtype=torch.int8)
    rows[..., :D_acc] = torch.randint(-5, 13, (E, C, D_acc), generator=gen, dtype=torch.int8)
    owner = torch.randint(0, N + 1, (E, C), generator=gen, dtype=torch.int8)
    off_obs, rows, owner = off_obs.cuda(), rows.cuda(), owner.cuda()
    crow = _common_row(D_acc, s_acc, O).cuda()
    ctr = torch.tensor([24], dtype=torch.int64, device="cuda")
    fo, fa = ppo.ActFrag(off, s_off), ppo.ActFrag(acc, s_acc, crow)
    fo.build(off)
    fa.build(acc)
    for rb in (0, 64):
        o1, l1 = off.act(off_obs, N * L, 55, 1, offset_dev=ctr, replica_base=rb)
        a1, al1 = acc.act_compact(rows, owner, N * C, 55, 3, crow, offset_dev=ctr, replica_base=rb)
        for of, af in ((None, None), (fo, fa)):
            out = dict(core_action=torch.empty_like(o1), core_logprob=torch.empty_like(l1))
            a2, al2 = torch.empty_like(a1), torch.empty_like(al1)
            ppo.act_round_free(off, None, off_obs, acc, rows, owner, crow, C, 55, 1, 3, out, a2, al2, offset_dev=ctr,
                               core_frag=of, acc_frag=af, replica_base=rb)
            assert torch.equal(out["core_action"], o1) and torch.equal(a2, a1), (rb, of is None)
            assert torch.equal(out["core_logprob"].view(torch.int32), l1.view(torch.int32))
            assert torch.equal(al2.view(torch.int32), al1.view(torch.int32))


@pytest.mark.parametrize("N,C,L,O,E", [(8, 8, 3, 24, 2048), (4, 4, 3, 12, 301), (16, 16, 3, 48, 97)])
def test_act_round_free_matches_separate_calls(ms, N, C, L, O, E):
    """ms_act_round_free (offer units + compact acceptor units in one launch; the paired kernel for
    cfg3's shapes, two launches otherwise) == ms_offer_act_free + ms_policy_act_compact, bit for bit."""
    ppo = _ppo(ms)
    torch.manual_seed(11)
    D_off, A_off, D_acc, A_acc = 2 * C + 2, C + 1, 3 + 2 * O, O + 1
    s_off, s_acc = (D_off + 3) & ~3, (D_acc + 3) & ~3
    core = ppo.GroupedActorCritic(N, D_off, A_off).cuda()
    price = ppo.GroupedActorCritic(N, 4, 13).cuda()
    acc = ppo.GroupedActorCritic(N, D_acc, A_acc).cuda()
    gen = torch.Generator().manual_seed(12)
    off_obs = torch.zeros((E, N * L, s_off), dtype=torch.int8)
    off_obs[..., :D_off] = torch.randint(-1, 13, (E, N * L, D_off), generator=gen, dtype=torch.int8)
    rows = torch.zeros((E, C, s_acc), dtype=torch.int8)
    rows[..., :D_acc] = torch.randint(-5, 13, (E, C, D_acc), generator=gen, dtype=torch.int8)
    owner = torch.randint(0, N + 1, (E, C), generator=gen, dtype=torch.int8)
    off_obs, rows, owner = off_obs.cuda(), rows.cuda(), owner.cuda()
    crow = _common_row(D_acc, s_acc, O).cuda()
    ctr = torch.tensor([40], dtype=torch.int64, device="cuda")

    def outs():
        d = "cuda"
        return dict(core_action=torch.empty((E, N * L), dtype=torch.int8, device=d),
                    core_logprob=torch.empty((E, N * L), device=d),
                    price_state=torch.empty((E, N * L, 4), dtype=torch.int8, device=d),
                    price_action=torch.empty((E, N * L), dtype=torch.int8, device=d),
                    price_logprob=torch.empty((E, N * L), device=d),
                    env_price=torch.empty((E, N * L), dtype=torch.int8, device=d))
    o1, o2 = outs(), outs()
    ppo.offer_act_free(core, price, off_obs, C, 77, 5, o1, offset_dev=ctr)
    a1, l1 = acc.act_compact(rows, owner, N * C, 77, 7, crow, offset_dev=ctr)
    a2 = torch.empty_like(a1)
    l2 = torch.empty_like(l1)
    ppo.act_round_free(core, price, off_obs, acc, rows, owner, crow, C, 77, 5, 7, o2, a2, l2, offset_dev=ctr)
    for k in o1:
        assert torch.equal(o1[k].view(torch.int8), o2[k].view(torch.int8)), k
    assert torch.equal(a1, a2)
    assert torch.equal(l1.view(torch.int32), l2.view(torch.int32))
    # with ms_act_prepare's weight fragments (and the acceptors' common-row table): bit-identical; a
    # block made for another row shape is ignored (its header does not match the call)
    fc, fa = ppo.ActFrag(core, s_off), ppo.ActFrag(acc, s_acc, crow)
    fc.build(core)
    fa.build(acc)
    wrong = ppo.ActFrag(acc, s_acc + 32, crow)  # another layer-1 k-step count
    wrong.build(acc)
    for core_frag, acc_frag in ((fc, fa), (None, fa), (fc, None), (None, wrong)):
        o4 = outs()
        a4, l4 = torch.empty_like(a1), torch.empty_like(l1)
        ppo.act_round_free(core, price, off_obs, acc, rows, owner, crow, C, 77, 5, 7, o4, a4, l4, offset_dev=ctr,
                           core_frag=core_frag, acc_frag=acc_frag)
        for k in o1:
            assert torch.equal(o1[k].view(torch.int8), o4[k].view(torch.int8)), (k, core_frag, acc_frag)
        assert torch.equal(a1, a4)
        assert torch.equal(l1.view(torch.int32), l4.view(torch.int32))
    a5, l5 = acc.act_compact(rows, owner, N * C, 77, 7, crow, offset_dev=ctr, frag=fa)
    assert torch.equal(a1, a5) and torch.equal(l1.view(torch.int32), l5.view(torch.int32))
    # unit-major price outputs (a [U][T][E] ring at round t = 1 of T = 3, as the trainer keeps them):
    # the same values at (u, t, e); env_price stays [E][U]
    T, t, U = 3, 1, N * L
    ring = dict(price_state=torch.zeros((U, T, E, 4), dtype=torch.int8, device="cuda"),
                price_action=torch.zeros((U, T, E), dtype=torch.int8, device="cuda"),
                price_logprob=torch.zeros((U, T, E), device="cuda"))
    for fn in ("offer_act_free", "act_round_free"):
        o3 = outs()
        o3.update({k: v[:, t] for k, v in ring.items()})
        if fn == "offer_act_free":
            ppo.offer_act_free(core, price, off_obs, C, 77, 5, o3, offset_dev=ctr, price_unit_stride=T * E)
        else:
            ppo.act_round_free(core, price, off_obs, acc, rows, owner, crow, C, 77, 5, 7, o3, a2, l2, offset_dev=ctr,
                               price_unit_stride=T * E)
        for k in ring:
            got = ring[k][:, t].movedim(0, 1).contiguous()  # [E][U](, 4)
            assert torch.equal(got.view(torch.int8), o1[k].view(torch.int8)), (fn, k)
            assert not ring[k][:, t - 1].any() and not ring[k][:, t + 1].any(), (fn, k)  # other rounds untouched
        for k in ("core_action", "core_logprob", "env_price"):
            assert torch.equal(o3[k].view(torch.int8), o1[k].view(torch.int8)), (fn, k)
        for v in ring.values():
            v.zero_()


@pytest.mark.parametrize("name", ["cfg3", "cfg4"])
def test_price_table_matches_computed_price_chooser(ms, name):
    """The price chooser sampling from its table (ms_price_table_build + ms_act_round_free) ==
    computing the net per row, bit for bit, including rows outside the table (injected bytes)."""
    ppo = _ppo(ms)
    abi = importlib.import_module("marl-scheduling_amd.abi")
    cfg = abi.named_config(name)
    s = abi.config_shape(cfg)
    N, C, L, O = s["N"], s["C"], s["L"], s["O"]
    E = 1500
    torch.manual_seed(13)
    D_off, A_off, D_acc, A_acc = 2 * C + 2, C + 1, 3 + 2 * O, O + 1
    s_off, s_acc = (D_off + 3) & ~3, (D_acc + 3) & ~3
    core = ppo.GroupedActorCritic(N, D_off, A_off).cuda()
    price = ppo.GroupedActorCritic(N, 4, s["price_actions"]).cuda()
    acc = ppo.GroupedActorCritic(N, D_acc, A_acc).cuda()
    gen = torch.Generator().manual_seed(14)
    off_obs = torch.zeros((E, N * L, s_off), dtype=torch.int8)
    prio = torch.randint(-1, max(cfg.job_priority[: cfg.n_kinds]) + 1, (E, N * L, C + 1), generator=gen)
    rem = torch.randint(-1, max(cfg.job_length[: cfg.n_kinds]) + 1, (E, N * L, C + 1), generator=gen)
    off_obs[..., 0:D_off:2] = prio.to(torch.int8)
    off_obs[..., 1:D_off:2] = rem.to(torch.int8)
    odd = torch.rand((E, N * L), generator=gen) < 0.01  # a few rows with a byte outside the table
    off_obs[odd, 1] = 40
    off_obs[odd, 2 * C + 1] = 41
    rows = torch.zeros((E, C, s_acc), dtype=torch.int8)
    rows[..., :D_acc] = torch.randint(-5, 13, (E, C, D_acc), generator=gen, dtype=torch.int8)
    owner = torch.randint(0, N + 1, (E, C), generator=gen, dtype=torch.int8)
    off_obs, rows, owner = off_obs.cuda(), rows.cuda(), owner.cuda()
    crow = _common_row(D_acc, s_acc, O).cuda()
    table = ppo.PriceTable(cfg, price)
    table.build(price)

    def outs():
        d = "cuda"
        return dict(core_action=torch.empty((E, N * L), dtype=torch.int8, device=d),
                    core_logprob=torch.empty((E, N * L), device=d),
                    price_state=torch.empty((E, N * L, 4), dtype=torch.int8, device=d),
                    price_action=torch.empty((E, N * L), dtype=torch.int8, device=d),
                    price_logprob=torch.empty((E, N * L), device=d),
                    env_price=torch.empty((E, N * L), dtype=torch.int8, device=d))
    res = []
    for tab in (None, table):
        o = outs()
        a = torch.empty((E, N * C), dtype=torch.int8, device="cuda")
        lp = torch.empty((E, N * C), device="cuda")
        ppo.act_round_free(core, price, off_obs, acc, rows, owner, crow, C, 5, 1, 3, o, a, lp, price_table=tab)
        res.append((o, a, lp))
    for k in res[0][0]:
        assert torch.equal(res[0][0][k].view(torch.int8), res[1][0][k].view(torch.int8)), k
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])
    # the table covers the dummy row and most sampled rows
    assert (res[1][0]["price_state"] == -5).all(-1).any()


def test_trainer_compact_matches_materialised(ms):
    """The trainer on compact acceptor rings (the env emits core rows + owners, the act and gradient
    kernels read them) == the trainer on the materialised [N*C] rows, bit for bit over two PPO
    iterations (rings, actions, losses, weights)."""
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    trs = [tr_mod.Trainer.from_named("cfg3", n_envs=64, update_step=12, seed=5, device="cuda:0", compact=c)
           for c in (True, False)]
    assert trs[0].compact and not trs[1].compact
    for _ in range(2):
        outs = [t.iteration() for t in trs]
        for k in outs[0]:
            assert torch.equal(outs[0][k], outs[1][k]), k
    assert torch.equal(trs[0].acceptor_rows(), trs[1].acceptor_rows())
    assert torch.equal(trs[0].acc.actions, trs[1].acc.actions)
    for u0, u1 in zip(trs[0].units(), trs[1].units()):
        for k in importlib.import_module("marl-scheduling_amd.ppo").ACTOR_KEYS:
            assert torch.equal(getattr(u0.group.policy, k), getattr(u1.group.policy, k)), (u0.name, k)


def test_trainer_fused_matches_torch_update(ms):
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    trs = [tr_mod.Trainer.from_named("cfg3", n_envs=32, update_step=20, seed=4, device="cuda:0", fused=f)
           for f in (True, False)]
    out = [t.iteration() for t in trs]
    for name in out[0]:
        np.testing.assert_allclose(out[0][name].cpu().numpy(), out[1][name].cpu().numpy(), rtol=1e-4, atol=1e-5)
    for u0, u1 in zip(trs[0].units(), trs[1].units()):
        for k in importlib.import_module("marl-scheduling_amd.ppo").ACTOR_KEYS:
            np.testing.assert_allclose(getattr(u0.group.policy, k).detach().cpu().numpy(),
                                       getattr(u1.group.policy, k).detach().cpu().numpy(), rtol=1e-4, atol=1e-5)


def test_trainer_one_allreduce_per_update_step(ms):
    """The unit types' gradients of one (draw, epoch) step share one flattened all-reduce (§8(e)):
    cfg3 locally shared has 2 draws x K=1 for acceptor, core chooser and price chooser -> 2 calls
    carrying all three types' parameters, and the same result as the per-type order."""
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    trs = [tr_mod.Trainer.from_named("cfg3", n_envs=32, update_step=10, seed=6, device="cuda:0") for _ in range(2)]
    calls = []
    trs[0].world_size = 2  # route through the all-reduce hook without a process group
    trs[0]._allreduce = lambda ps: calls.append(sum(p.numel() for p in ps))
    out = [t.iteration() for t in trs]
    n_params = sum(p.numel() for u in trs[0].units() for p in u.group.policy.parameters())
    assert calls == [n_params, n_params]
    for name in out[0]:
        assert torch.equal(out[0][name], out[1][name])


@pytest.mark.parametrize("G,per_group,C,A2", [(8, 3, 8, 13), (2, 3, 2, 11), (1, 48, 16, 11)])
def test_offer_act_free_matches_reference(ms, G, per_group, C, A2):
    """FreePriceOfferPPO.selectAction (PPOmodules.py:312-332) fused: core chooser, price input, price chooser."""
    ppo = _ppo(ms)
    torch.manual_seed(2)
    D, A = 2 * C + 2, C + 1
    stride = (D + 3) & ~3
    core = ppo.GroupedActorCritic(G, D, A)
    price = ppo.GroupedActorCritic(G, 4, A2)
    E, U = 257, G * per_group
    gen = torch.Generator().manual_seed(3)
    obs = torch.zeros((E, U, stride), dtype=torch.int8)
    obs[..., :D] = torch.randint(-1, 13, (E, U, D), generator=gen, dtype=torch.int8)
    u = torch.rand((2, E, U), generator=gen)
    dev = "cuda"
    out = dict(core_action=torch.empty((E, U), dtype=torch.int8, device=dev),
               core_logprob=torch.empty((E, U), device=dev),
               price_state=torch.empty((E, U, 4), dtype=torch.int8, device=dev),
               price_action=torch.empty((E, U), dtype=torch.int8, device=dev),
               price_logprob=torch.empty((E, U), device=dev),
               env_price=torch.empty((E, U), dtype=torch.int8, device=dev))
    ppo.offer_act_free(core.cuda(), price.cuda(), obs.cuda(), C, 0, 0, out, uniforms=u.cuda())
    out = {k: v.cpu() for k, v in out.items()}
    for g in range(G):
        sl = slice(g * per_group, (g + 1) * per_group)
        cf = {k: getattr(core, k)[g].detach().cpu() for k in ppo.ACTOR_KEYS}
        pf = {k: getattr(price, k)[g].detach().cpu() for k in ppo.ACTOR_KEYS}
        x = obs[:, sl, :D].float()
        ra, rlp, _ = act_reference(cf, x, u[0][:, sl])
        ga = out["core_action"][:, sl].long()
        ok = ga == ra
        assert ok.float().mean() > 0.999
        np.testing.assert_allclose(out["core_logprob"][:, sl][ok].numpy(), rlp[ok].numpy(), rtol=1e-5, atol=2e-6)
        # price chooser input from the device's own core action
        idx = (2 * ga).unsqueeze(-1) + torch.arange(2)
        pin = torch.cat((torch.gather(x, 2, idx), x[..., 2 * C:2 * C + 2]), -1)
        pin = torch.where((ga == 0).unsqueeze(-1), torch.full_like(pin, -5.0), pin)
        assert torch.equal(out["price_state"][:, sl].float(), pin)
        pa, plp, _ = act_reference(pf, pin, u[1][:, sl])
        gp = out["price_action"][:, sl].long()
        okp = gp == pa
        assert okp.float().mean() > 0.999
        np.testing.assert_allclose(out["price_logprob"][:, sl][okp].numpy(), plp[okp].numpy(), rtol=1e-5, atol=2e-6)
        want_env = torch.where(ga == 0, torch.full_like(gp, -5), gp)
        assert torch.equal(out["env_price"][:, sl].long(), want_env)


def test_trainer_graph_replay_matches_eager(ms):
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    trs = [tr_mod.Trainer.from_named("cfg3", n_envs=48, update_step=16, seed=9, device="cuda:0", use_graph=g)
           for g in (True, False)]
    kept = ([], [])  # every iteration's losses as a caller keeps them (no aliasing)
    last = ([], [])
    for _ in range(4):
        for i, t in enumerate(trs):
            kept[i].append(t.iteration())
            last[i].append({u.name: u.group.last_losses for u in t.units()})
    for it in range(4):  # earlier graphed iterations' losses were not overwritten by later replays
        for k in kept[0][it]:
            assert torch.equal(kept[0][it][k], kept[1][it][k]), (it, k)
            for a, b in zip(last[0][it][k], last[1][it][k]):
                assert torch.equal(a, b), (it, k)
    assert not torch.equal(kept[0][1]["acceptor"], kept[0][3]["acceptor"])
    assert torch.equal(trs[0].acceptor_rows(), trs[1].acceptor_rows())
    assert trs[0].env.round == trs[1].env.round == 64


def test_trainer_two_stream_rollout(ms):
    """rollout_streams=2: the replicas split in two parts stepped on two HIP streams. Every replica keeps
    its seed and its Philox rows (ms_mlp_params.row_base), so the split rollout is bit-identical to the
    unsplit trainer's, and the split graph replay equals the split eager rollout."""
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    E, T = 64, 12
    mk = lambda streams, g: tr_mod.Trainer.from_named("cfg3", n_envs=E, update_step=T, seed=4, device="cuda:0",
                                                      use_graph=g, rollout_streams=streams)
    one, two_g, two_e = mk(1, False), mk(2, True), mk(2, False)
    one.rollout()
    two_g.rollout()
    two_e.rollout()
    torch.cuda.synchronize()
    assert torch.equal(one.acceptor_rows(), two_e.acceptor_rows())
    assert torch.equal(one.off_obs, two_e.off_obs)
    for u in ("acc", "off", "price"):
        assert torch.equal(getattr(one, u).actions, getattr(two_e, u).actions), u
        assert torch.equal(getattr(one, u).logprobs, getattr(two_e, u).logprobs), u
        assert torch.equal(getattr(one, u).rewards, getattr(two_e, u).rewards), u
    for _ in range(2):  # graph capture happened in the first rollout; replays from here
        two_g.rollout()
        two_e.rollout()
    assert torch.equal(two_g.acceptor_rows(), two_e.acceptor_rows())
    for name in ("off_obs", "price_obs"):
        assert torch.equal(getattr(two_g, name), getattr(two_e, name)), name
    for u in ("acc", "off", "price"):
        assert torch.equal(getattr(two_g, u).actions, getattr(two_e, u).actions), u
        assert torch.equal(getattr(two_g, u).rewards, getattr(two_e, u).rewards), u
    assert two_g.env.round == two_e.env.round == 3 * T
    assert two_g.flags() == 0 and two_e.flags() == 0
    losses = [t.update() for t in (two_g, two_e)]
    for k in losses[0]:
        assert torch.equal(losses[0][k], losses[1][k]), k


def test_hip_adam_matches_torch_adam(ms):
    """ms_adam_step (HipAdam) against torch.optim.Adam with the actor / critic param groups of
    PPO.__init__ (PPOmodules.py:100-105), over several steps with changing gradients."""
    ppo = _ppo(ms)
    gen = torch.Generator().manual_seed(3)
    shapes = [(8, 16, 51), (8, 16), (8, 16, 16), (8, 25, 16), (8, 1, 16), (8, 1)]
    init = [torch.randn(s, generator=gen) for s in shapes]
    p_ref = [t.clone().cuda().requires_grad_(True) for t in init]
    p_hip = [t.clone().cuda().requires_grad_(True) for t in init]
    groups = lambda ps: [{"params": ps[:4], "lr": 0.003}, {"params": ps[4:], "lr": 0.01}]
    ref = torch.optim.Adam(groups(p_ref))
    hip = ppo.HipAdam(groups(p_hip))
    for step in range(6):
        grads = [torch.randn(s, generator=gen).cuda() * (10.0 ** (step - 3)) for s in shapes]
        for p, g in zip(p_ref, grads):
            p.grad = g.clone()
        for p, g in zip(p_hip, grads):
            p.grad = g.clone()
        ref.step()
        hip.step()
        for i, (a, b) in enumerate(zip(p_hip, p_ref)):
            np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().cpu().numpy(), rtol=2e-6, atol=1e-7,
                                       err_msg="tensor %d step %d" % (i, step))
        for i, (a, b) in enumerate(zip(p_hip, p_ref)):
            st_h, st_r = hip.state[a], ref.state[b]
            np.testing.assert_allclose(st_h["exp_avg_sq"].cpu().numpy(), st_r["exp_avg_sq"].cpu().numpy(), rtol=2e-6,
                                       atol=0)


def test_unit_returns_of_several_draws_feed_the_gradient(ms):
    """One ms_unit_returns launch for two draws (unit_of_group concatenated) read through
    ms_ppo_batch.returns_ld gives the same gradient as separate per-draw returns."""
    ppo = _ppo(ms)
    G, T, E, U, D, stride, A = 4, 12, 40, 12, 18, 20, 9
    states, actions, old_lp, _ = _rand_batch(G, T, E, U, D, stride, A, 9)
    gen = torch.Generator().manual_seed(5)
    rew = torch.randint(-5, 9, (T, E, U), generator=gen).float().cuda()
    draws = [torch.randint(0, U, (G,), generator=gen).to(torch.int32).cuda() for _ in range(2)]
    both = torch.cat(draws)
    ret_both = ppo.unit_returns(rew, both, 0.5)
    for d, sel in enumerate(draws):
        torch.manual_seed(7)
        g1 = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.5, 0.2, 1, device="cuda")
        torch.manual_seed(7)
        g2 = ppo.PPOGroup(G, D, A, 0.003, 0.01, 0.5, 0.2, 1, device="cuda")
        ret_one = ppo.unit_returns(rew, sel, 0.5)
        torch.testing.assert_close(ret_both[:, :, d * G:(d + 1) * G], ret_one, rtol=0, atol=0)
        l1 = g1.update_fused(states.cuda(), actions.cuda(), old_lp.cuda(), ret_one, sel, T, E)
        l2 = g2.update_fused(states.cuda(), actions.cuda(), old_lp.cuda(), ret_both.view(-1)[d * G:], sel, T, E,
                             returns_ld=2 * G)
        torch.testing.assert_close(l1[0], l2[0], rtol=0, atol=0)
        for k in ppo.ACTOR_KEYS + ppo.CRITIC_KEYS:
            torch.testing.assert_close(getattr(g1.policy, k), getattr(g2.policy, k), rtol=0, atol=0)


def test_trainer_price_unit_major_matches(ms, monkeypatch):
    """MS_PRICE_UNIT_MAJOR=1 (price chooser rings [U][T][E], ms_act_round_free's price_unit_stride and
    ms_ppo_batch.unit_stride): the same rollout and update, bit for bit."""
    tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
    trs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("MS_PRICE_UNIT_MAJOR", flag)
        tr = tr_mod.Trainer.from_named("cfg3", n_envs=96, update_step=10, seed=6, device="cuda:0")
        assert tr.price_unit_major == (flag == "1")
        losses = [tr.iteration() for _ in range(2)]
        torch.cuda.synchronize()
        trs.append((tr, losses))
    (a, la), (b, lb) = trs
    assert torch.equal(a.price_obs, b.price_obs) and torch.equal(a.price.actions, b.price.actions)
    assert torch.equal(a.price.logprobs, b.price.logprobs) and torch.equal(a.off.actions, b.off.actions)
    for x, y in zip(la, lb):
        for k in x:
            assert torch.equal(x[k], y[k]), k
    for k in ("w1", "b3"):
        assert torch.equal(getattr(a.price.group.policy, k), getattr(b.price.group.policy, k)), k
