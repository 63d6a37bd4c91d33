"""Branching DQN on compact observations (§8(f) rows 1 and 4, BASELINE cfg5): the env kernel's compact
acceptor outputs and their regeneration bit-exact against the full rows, the structured layer 1
against the dense BranchingQNetwork, and update_policy against the torch restatement of
BranchingDQNModules.py (oracle/bdqn_ref.py)."""
import importlib

import numpy as np
import pytest
import torch

from oracle.bdqn_ref import RefBranchingQNetwork, layer1_compact_reference, update_policy_reference
from tests.drivers import offer_counts_from_obs, random_actions

pytestmark = pytest.mark.gpu


def _bdqn():
    return importlib.import_module("marl-scheduling_amd.bdqn")


@pytest.mark.parametrize("kw", [dict(n_agents=5, n_cores=6, collection_length=3, priorities=[3, 10], lengths=[6, 3],
                                     fix_prices=[2, 7], probabilities=[0.8, 0.2]),
                                dict(n_agents=4, n_cores=3, collection_length=2, priorities=[2, 4, 8],
                                     lengths=[5, 5, 3], probabilities=[0.5, 0.25, 0.25], free_prices=True)])
def test_compact_observations_regenerate_the_rows(ms, kw):
    abi = ms.abi
    cfg = abi.make_config(**kw)
    s = abi.config_shape(cfg)
    N, C, L, O = s["N"], s["C"], s["L"], s["O"]
    E, T = 40, 60
    env = ms.BatchedEnv(cfg, E, seed=3)
    dev = env.device
    full = env.obs_buffers()
    comp = env.compact_obs_buffers()
    env.reset(dict(full, **{k: comp[k] for k in ("core_rows", "core_owner")}))
    rng = np.random.default_rng(0)
    free = bool(cfg.free_prices)
    M = T + 1
    rows = torch.zeros((M, E, C, s["acc_obs_stride"]), dtype=torch.int8, device=dev)
    owners = torch.zeros((M, E, C), dtype=torch.int8, device=dev)
    pairs = torch.zeros((M, E, N, L, 2), dtype=torch.int8, device=dev)
    aggs = []
    for t in range(M):
        rows[t].copy_(comp["core_rows"])
        owners[t].copy_(comp["core_owner"])
        pairs[t].copy_(full["offer"][..., 2 * C:2 * C + 2])
        acc_h = full["acceptor"].cpu().numpy()
        cr, co = comp["core_rows"].cpu().numpy(), comp["core_owner"].cpu().numpy()
        st = env.export_state()
        assert np.array_equal(co, st["core_owner"].reshape(E, C))
        foreign = np.array([0, -1, -1] + [-2] * (2 * O) + [0] * (s["acc_obs_stride"] - s["acc_obs_dim"]), np.int8)
        for a in range(N):
            want = np.where((co == a + 1)[..., None], cr, foreign[None, None, :])
            assert np.array_equal(acc_h[:, a], want), (t, a)
        agg = {k: v.clone() for k, v in env.aggregate_obs(full, kinds=("acceptor", "offer")).items()}
        aggs.append(agg)
        if t == T:
            break
        counts = [offer_counts_from_obs(acc_h[e, :, :, : s["acc_obs_dim"]], O) for e in range(E)]
        acts = [random_actions(rng, counts[e], N, C, L, O, free, s["price_actions"] - 1) for e in range(E)]
        acc = torch.tensor(np.stack([x[0] for x in acts]), dtype=torch.int8, device=dev)
        off = torch.tensor(np.stack([x[1] for x in acts]), dtype=torch.int8, device=dev)
        pr = torch.tensor(np.stack([x[2] for x in acts]), dtype=torch.int8, device=dev) if free else None
        env.step(acc, off, pr, obs=dict(full, **{k: comp[k] for k in ("core_rows", "core_owner")}))
    # regenerate random (record, agent) samples from the ring and compare with the aggregated rows
    g = torch.Generator().manual_seed(1)
    n = 500
    frame = torch.randint(0, M * E, (n,), generator=g)
    agent = torch.randint(0, N, (n,), generator=g, dtype=torch.int32)
    ra, ro = env.regen_agent_rows(rows.view(-1, C, s["acc_obs_stride"]), owners.view(-1, C), pairs.view(-1, N, L, 2),
                                  frame.to(dev), agent.to(dev))
    ra, ro = ra.cpu(), ro.cpu()
    for b in range(n):
        t, e, a = int(frame[b]) // E, int(frame[b]) % E, int(agent[b])
        assert torch.equal(ra[b], aggs[t]["acceptor"][e, a].cpu()), b
        assert torch.equal(ro[b], aggs[t]["offer"][e, a].cpu()), b


def _cfg5_compact(ms, E, steps=30, seed=5):
    abi = ms.abi
    cfg = abi.named_config("cfg5")
    s = abi.config_shape(cfg)
    N, C = s["N"], s["C"]
    env = ms.BatchedEnv(cfg, E, seed=seed)
    comp = env.compact_obs_buffers()
    env.reset(comp)
    rng = np.random.default_rng(2)
    for _ in range(steps):
        acc = torch.tensor(rng.integers(0, s["O"] + 1, (E, N, C)), dtype=torch.int8, device=env.device)
        off = torch.tensor(rng.integers(0, C + 1, (E, N, s["L"])), dtype=torch.int8, device=env.device)
        pr = torch.tensor(rng.integers(0, s["price_actions"], (E, N, s["L"])), dtype=torch.int8, device=env.device) \
            if cfg.free_prices else None
        env.step(acc, off, pr, obs=comp)
    return env, comp, s


def _dense_rows(env, comp, s):
    N, C = s["N"], s["C"]
    E = comp["core_owner"].shape[0]
    frame = torch.arange(E, device=env.device).repeat_interleave(N)
    agent = torch.arange(N, dtype=torch.int32, device=env.device).repeat(E)
    pairs = comp["offer"][..., 2 * C:2 * C + 2].contiguous()
    return env.regen_agent_rows(comp["core_rows"], comp["core_owner"], pairs, frame, agent)


def test_structured_layer1_matches_dense(ms):
    """ms_bdqn_layer1_compact (exact bf16 products, f32 sums, owners' rows added in core order) against
    the dense Linear(C * D_acc, 128) of the regenerated aggregated acceptor rows (fp32 torch), and the
    torch algebra of oracle/bdqn_ref.layer1_compact_reference; bit-identical on a repeat."""
    bdqn = _bdqn()
    E = 64
    env, comp, s = _cfg5_compact(ms, E)
    N, C, D = s["N"], s["C"], s["acc_obs_dim"]
    torch.manual_seed(0)
    net = bdqn.BranchingQ(C * D, C, s["O"] + 1).cuda()
    actor = bdqn.HipActor(net, D, C, "cuda", compact=True)
    actor.prepare()
    h_k = actor.layer1_compact(comp["core_rows"], comp["core_owner"], N)
    h_k2 = actor.layer1_compact(comp["core_rows"], comp["core_owner"], N)
    assert torch.equal(h_k, h_k2)
    with torch.no_grad():
        ra, _ = _dense_rows(env, comp, s)
        x = ra[:, : C * D].float()
        h_d = torch.nn.functional.linear(x.cpu().double(), net.w1.detach().cpu().double(),
                                         net.b1.detach().cpu().double())
        h_r = layer1_compact_reference(net.w1, net.b1, comp["core_rows"], comp["core_owner"], N, D)
    scale = h_d.abs().max().item()
    assert (h_k.cpu().double() - h_d).abs().max().item() <= 1e-5 * scale
    assert (h_r.cpu().double() - h_d).abs().max().item() <= 1e-5 * scale
    assert (comp["core_owner"] > 0).sum().item() > 0  # the structured path saw agent-owned cores


def _check_greedy(q, got, gap=1e-5):
    """got [B, ac] int8 vs the first argmax of q [B, ac, n] (fp32): equal wherever the best q is ahead
    of the second by more than gap of the q scale (elsewhere the two are within f32 rounding)."""
    top2 = q.topk(2, dim=2).values
    scale = q.abs().max().item()
    clear = (top2[..., 0] - top2[..., 1]) > gap * scale
    want = q.argmax(2)
    assert clear.float().mean().item() > 0.95
    assert torch.equal(got.long()[clear], want[clear])
    return (got.long() == want).float().mean().item()


@pytest.mark.parametrize("role", ["acc", "off", "price"])
def test_act_kernel_is_the_argmax_of_q(ms, role):
    """ms_bdqn_act (trunk + value + advantage heads + per-branch q and first argmax, epsilon-greedy)
    against q = value + adv - mean(adv) of the reference BranchingQNetwork (oracle/bdqn_ref.py,
    BranchingDQNModules.py:75-101, fp32 on the CPU); explored rows take the given random actions."""
    bdqn = _bdqn()
    E = 96
    env, comp, s = _cfg5_compact(ms, E, steps=25, seed=7)
    N, C, L, D = s["N"], s["C"], s["L"], s["acc_obs_dim"]
    dims = env.aggregated_dims()
    ra, ro = _dense_rows(env, comp, s)
    if role == "acc":
        obs, ac, n = C * D, C, s["O"] + 1
    else:
        obs, ac, n = dims["offer"][0], L, (C + 1 if role == "off" else s["price_actions"])
    torch.manual_seed(11)
    net = bdqn.BranchingQ(obs, ac, n).cuda()
    actor = bdqn.HipActor(net, D if role == "acc" else obs, C if role == "acc" else 1, "cuda", compact=role == "acc")
    actor.prepare()
    rows = E * N
    g = torch.Generator(device="cuda").manual_seed(3)
    explore = (torch.rand((rows,), generator=g, device="cuda") < 0.3).to(torch.uint8)
    rnd = torch.randint(0, n, (rows, ac), generator=g, device="cuda").to(torch.int8)
    if role == "acc":
        h1 = actor.layer1_compact(comp["core_rows"], comp["core_owner"], N)
        got = actor.act(h1=h1, explore=explore, rand_action=rnd)
        greedy = actor.act(h1=h1)
        x = ra[:, :obs].float()
    else:
        got = actor.act(x=ro, explore=explore, rand_action=rnd)
        greedy = actor.act(x=ro)
        x = ro[:, :obs].float()
    assert torch.equal(got, actor.act(h1=h1, explore=explore, rand_action=rnd) if role == "acc"
                       else actor.act(x=ro, explore=explore, rand_action=rnd))  # deterministic
    ref = RefBranchingQNetwork(obs, ac, n)
    ref.load_stacked({k: getattr(net, k).detach().cpu() for k in bdqn.KEYS})
    with torch.no_grad():
        q = ref(x.cpu())
    agree = _check_greedy(q, greedy.cpu())
    assert agree > 0.995
    ex = explore.cpu().bool()
    assert torch.equal(got.cpu()[ex], rnd.cpu()[ex])
    assert torch.equal(got.cpu()[~ex], greedy.cpu()[~ex])


@pytest.mark.parametrize("n", [17, 33, 50, 65, 100])
def test_act_kernel_masks_padded_action_tiles(ms, n):
    """Branch widths whose tile count is not an instantiated NMT (n = 17: NMT 3 for 2 tiles; 50, 65,
    100: NMT 7 for 4..6 tiles; 33 is exact) on int8 rows (layer 1 in the kernel): the zero-padded
    rows past n join neither the mean nor the argmax, so every action is < n and the greedy ones are
    the first argmax of the fp32 reference's q (BranchingDQNModules.py:88-101). The advantage biases
    are shifted so the mean advantage is negative, where a padded row would win."""
    bdqn = _bdqn()
    obs, ac, rows = 40, 3, 3000
    torch.manual_seed(n)
    net = bdqn.BranchingQ(obs, ac, n).cuda()
    with torch.no_grad():
        net.ba.sub_(0.5)
    actor = bdqn.HipActor(net, obs, 1, "cuda")
    actor.prepare()
    g = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randint(-5, 14, (rows, 40), generator=g, device="cuda").to(torch.int8)
    got = actor.act(x=x)
    assert int(got.min()) >= 0 and int(got.max()) < n
    ref = RefBranchingQNetwork(obs, ac, n)
    ref.load_stacked({k: getattr(net, k).detach().cpu() for k in bdqn.KEYS})
    with torch.no_grad():
        q = ref(x.cpu().float())
    assert _check_greedy(q, got.cpu()) > 0.995


def test_act_compact_equals_layer1_then_act(ms):
    """ms_bdqn_act_compact (the owned cores' P rows summed inside the act kernel) == ms_bdqn_layer1_compact
    followed by ms_bdqn_act on its h1, bit for bit, greedy and epsilon-greedy."""
    bdqn = _bdqn()
    E = 80
    env, comp, s = _cfg5_compact(ms, E, steps=9, seed=5)
    N, C, D = s["N"], s["C"], s["acc_obs_dim"]
    torch.manual_seed(13)
    net = bdqn.BranchingQ(C * D, C, s["O"] + 1).cuda()
    actor = bdqn.HipActor(net, D, C, "cuda", compact=True)
    actor.prepare()
    rows = E * N
    g = torch.Generator(device="cuda").manual_seed(9)
    explore = (torch.rand((rows,), generator=g, device="cuda") < 0.3).to(torch.uint8)
    rnd = torch.randint(0, net.n, (rows, C), generator=g, device="cuda").to(torch.int8)
    h1 = actor.layer1_compact(comp["core_rows"], comp["core_owner"], N)
    for ex, rn in ((None, None), (explore, rnd)):
        want = actor.act(h1=h1, explore=ex, rand_action=rn)
        got = actor.act_compact(comp["core_rows"], comp["core_owner"], N, explore=ex, rand_action=rn)
        assert torch.equal(got, want)
    assert (comp["core_owner"] > 0).sum().item() > 0


def test_update_matches_reference(ms):
    bdqn = _bdqn()
    torch.manual_seed(3)
    obs, ac, n, B = 70, 3, 33, 128
    cfg = bdqn.BDQNConfig(target_net_update_freq=2)
    role = bdqn.BranchingRole(obs, ac, n, cfg, "cuda")
    ref_q, ref_t = RefBranchingQNetwork(obs, ac, n), RefBranchingQNetwork(obs, ac, n)
    ref_q.load_stacked({k: getattr(role.q, k).detach().cpu() for k in bdqn.KEYS})
    ref_t.load_stacked({k: getattr(role.target, k).detach().cpu() for k in bdqn.KEYS})
    adam = torch.optim.Adam(ref_q.parameters(), lr=1e-4)
    g = torch.Generator().manual_seed(4)
    for step in range(3):
        s = torch.randint(-5, 13, (B, obs), generator=g).float()
        s1 = torch.randint(-5, 13, (B, obs), generator=g).float()
        a = torch.randint(0, n, (B, ac), generator=g)
        r = torch.randint(-30, 30, (B,), generator=g).float()
        m = (torch.rand((B,), generator=g) > 0.1).float()
        lg = role.update(s.cuda(), a.cuda(), r.cuda(), s1.cuda(), m.cuda())
        lr_ = update_policy_reference(ref_q, ref_t, adam, s, a, r, s1, m)
        assert abs(float(lg) - float(lr_)) <= 1e-4 * max(1.0, abs(float(lr_)))
        if step == 1:  # target_net_update_freq = 2
            ref_t.load_state_dict(ref_q.state_dict())
    want = ref_q.stacked()
    for k in bdqn.KEYS:
        np.testing.assert_allclose(getattr(role.q, k).detach().cpu().numpy(), want[k].detach().numpy(),
                                   rtol=1e-3, atol=1e-6)
    assert torch.equal(role.target.w1, role.q.w1.detach()) is False  # synced at update 2, updated once since


def test_graphed_update_equals_eager(ms):
    """BranchingRole(graph=True): the first update eager (on a side stream), then replays of the captured
    graph on the static inputs; with the target sync on the host. Same losses and weights as eager."""
    bdqn = _bdqn()
    obs, ac, n, B = 70, 3, 33, 128
    cfg = bdqn.BDQNConfig(target_net_update_freq=2)
    roles = []
    for graph in (False, True):
        torch.manual_seed(3)
        roles.append(bdqn.BranchingRole(obs, ac, n, cfg, "cuda", graph=graph))
    g = torch.Generator().manual_seed(4)
    for step in range(5):
        s = torch.randint(-5, 13, (B, obs), generator=g).float().cuda()
        s1 = torch.randint(-5, 13, (B, obs), generator=g).float().cuda()
        a = torch.randint(0, n, (B, ac), generator=g).cuda()
        r = torch.randint(-30, 30, (B,), generator=g).float().cuda()
        m = (torch.rand((B,), generator=g) > 0.1).float().cuda()
        l0, l1 = [ro.update(s, a, r, s1, m) for ro in roles]
        torch.testing.assert_close(l1, l0, rtol=1e-6, atol=1e-7)
    for k in bdqn.KEYS:
        torch.testing.assert_close(getattr(roles[1].q, k), getattr(roles[0].q, k), rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(getattr(roles[1].target, k), getattr(roles[0].target, k), rtol=1e-5, atol=1e-7)
    assert roles[1]._g is not None


def test_bdqn_trainer_cfg5(ms):
    bdqn = _bdqn()
    cfg = ms.abi.named_config("cfg5")
    b = bdqn.BDQNConfig(memory_frames=6, learning_starts=2, batch_size=64)
    tr = bdqn.BDQNTrainer(cfg, n_envs=48, bcfg=b, seed=1, episode_length=5)
    for _ in range(9):
        tr.step()
    assert tr.flags() == 0 and tr.env.round == 9 and tr.stored == 6
    assert set(tr.last_losses) >= {"acc", "off"}
    assert all(torch.isfinite(v) for v in tr.last_losses.values())


@pytest.mark.parametrize("obs,ac,n,B", [(70, 3, 33, 128), (6240, 32, 97, 128), (130, 32, 13, 77)])
def test_hip_update_matches_reference(ms, obs, ac, n, B):
    """ms_bdqn_update + HIP Adam (BranchingRole.hip_update) against the torch restatement of
    update_policy (oracle/bdqn_ref.py: the three forwards, the double-DQN target averaged over the
    branches, the broadcast MSE, the clamp, Adam) over three updates with a target sync after the
    second; the cfg5 acceptor shape (6240 inputs, 32 branches of 97) and a partial batch included."""
    bdqn = _bdqn()
    torch.manual_seed(3)
    cfg = bdqn.BDQNConfig(target_net_update_freq=2)
    role = bdqn.BranchingRole(obs, ac, n, cfg, "cuda")
    ref_q, ref_t = RefBranchingQNetwork(obs, ac, n), RefBranchingQNetwork(obs, ac, n)
    ref_q.load_stacked({k: getattr(role.q, k).detach().cpu() for k in bdqn.KEYS})
    ref_t.load_stacked({k: getattr(role.target, k).detach().cpu() for k in bdqn.KEYS})
    adam = torch.optim.Adam(ref_q.parameters(), lr=1e-4)
    g = torch.Generator().manual_seed(4)
    for step in range(3):
        s = torch.randint(-5, 13, (B, obs), generator=g, dtype=torch.int8)
        s1 = torch.randint(-5, 13, (B, obs), generator=g, dtype=torch.int8)
        a = torch.randint(0, n, (B, ac), generator=g)
        r = torch.randint(-30, 30, (B,), generator=g).float()
        m = (torch.rand((B,), generator=g) > 0.1).float()
        lg = role.hip_update(s.cuda(), s1.cuda(), a.to(torch.int8).cuda(), r.cuda(), m.cuda())
        role.count_update()
        lr_ = update_policy_reference(ref_q, ref_t, adam, s.float(), a, r, s1.float(), m)
        assert abs(float(lg) - float(lr_)) <= 1e-4 * max(1.0, abs(float(lr_))), (step, float(lg), float(lr_))
        if step == 1:  # target_net_update_freq = 2
            ref_t.load_state_dict(ref_q.state_dict())
    # Adam moves an element by about lr per step whatever its gradient's size, so an element whose
    # gradient sits at the f32 noise floor may move either way: at most 2 * lr * steps apart, and few
    def close(got, want, k):
        got, want = got.detach().cpu(), want.detach().cpu()
        off = ~torch.isclose(got, want, rtol=1e-3, atol=1e-6)
        assert int(off.sum()) <= max(2, off.numel() // 10000), (k, int(off.sum()))
        assert ((got - want)[off].abs() <= 2 * 1e-4 * 3 + 1e-6).all(), k

    want = ref_q.stacked()
    for k in bdqn.KEYS:
        close(getattr(role.q, k), want[k], k)
    tw = ref_t.stacked()
    for k in bdqn.KEYS:
        close(getattr(role.target, k), tw[k], k)


def test_hip_update_gradient_matches_autograd(ms):
    """One ms_bdqn_update's clamped gradient against torch autograd of the same update_policy loss
    (before Adam), element by element, and bit-identical on a repeat."""
    bdqn = _bdqn()
    obs, ac, n, B = 200, 4, 9, 128
    torch.manual_seed(5)
    cfg = bdqn.BDQNConfig(grad_clip=0.05)  # a small clamp: some elements hit it
    role = bdqn.BranchingRole(obs, ac, n, cfg, "cuda")
    with torch.no_grad():
        for k in bdqn.KEYS:  # a target different from the online net
            getattr(role.target, k).add_(0.01 * torch.randn_like(getattr(role.target, k)))
    g = torch.Generator().manual_seed(6)
    s = torch.randint(-5, 13, (B, obs), generator=g, dtype=torch.int8).cuda()
    s1 = torch.randint(-5, 13, (B, obs), generator=g, dtype=torch.int8).cuda()
    a = torch.randint(0, n, (B, ac), generator=g).cuda()
    r = torch.randint(-30, 30, (B,), generator=g).float().cuda()
    m = (torch.rand((B,), generator=g) > 0.1).float().cuda()
    # autograd of the loss on the current weights
    q = role.q
    current = q(s.float()).gather(2, a.unsqueeze(2)).squeeze(-1)
    with torch.no_grad():
        am = torch.argmax(q(s1.float()), dim=2)
        mx = role.target(s1.float()).gather(2, am.unsqueeze(2)).squeeze(-1).mean(1, keepdim=True)
    expected = r.view(-1, 1) + mx * 0.99 * m.view(-1, 1)
    loss = ((expected - current) ** 2).mean()
    want = torch.autograd.grad(loss, [getattr(q, k) for k in bdqn.KEYS])
    want = {k: w.clamp(-0.05, 0.05) for k, w in zip(bdqn.KEYS, want)}
    lr0 = role.opt.param_groups[0]["lr"]
    role.opt.param_groups[0]["lr"] = 0.0  # keep the weights: compare the gradient only
    l1 = role.hip_update(s, s1, a.to(torch.int8), r, m).clone()
    g1 = {k: getattr(q, k).grad.clone() for k in bdqn.KEYS}
    l2 = role.hip_update(s, s1, a.to(torch.int8), r, m).clone()
    role.opt.param_groups[0]["lr"] = lr0
    assert abs(float(l1) - float(loss)) <= 1e-5 * abs(float(loss))
    assert torch.equal(l1, l2)
    for k in bdqn.KEYS:
        assert torch.equal(g1[k], getattr(q, k).grad), k
        scale = want[k].abs().max().item() + 1e-12
        err = (g1[k] - want[k]).abs().max().item()
        assert err <= 1e-4 * scale + 1e-7, (k, err, scale)


def test_bdqn_trainer_hip_graph_equals_eager(ms):
    """The trainer's HIP learn step replayed from its captured graph == the same steps eager (same
    seeds, same draws), bit for bit, and the minibatch drawn without replacement."""
    bdqn = _bdqn()
    cfg = ms.abi.named_config("cfg5")
    trs = []
    for graph in (False, True):
        b = bdqn.BDQNConfig(memory_frames=5, learning_starts=2, batch_size=128, graph_updates=graph,
                            target_net_update_freq=3)
        trs.append(bdqn.BDQNTrainer(cfg, n_envs=40, bcfg=b, seed=2, episode_length=4))
    for _ in range(8):
        for tr in trs:
            tr.step()
        if trs[1].frame > b.learning_starts:  # a minibatch was drawn this frame
            sel = trs[1]._sel_host[0] * trs[1].N + trs[1]._sel_host[2]
            assert len(set(sel.tolist())) == 128
    assert trs[1]._learn_graph is not None
    for k in trs[0].roles:
        for key in bdqn.KEYS:
            assert torch.equal(getattr(trs[0].roles[k].q, key), getattr(trs[1].roles[k].q, key)), (k, key)
            assert torch.equal(getattr(trs[0].roles[k].target, key), getattr(trs[1].roles[k].target, key)), (k, key)
        assert torch.equal(trs[0].last_losses[k], trs[1].last_losses[k]), k
