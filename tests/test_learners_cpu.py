"""Host logic of the DQN / Branching-DQN learners and the metrics conversion on CPU (no kernels):
ReplayMemory.push semantics, the Branching DQN's structured layer 1 against the dense network on
synthetic compact observations, update_policy against its restatement, and episode_values on a
hand-filled accumulator."""
import importlib
import math

import numpy as np
import pytest
import torch

from oracle.bdqn_ref import RefBranchingQNetwork, update_policy_reference


def _mod(name):
    return importlib.import_module("marl-scheduling_amd." + name)


def test_replay_memories_push_on_cpu():
    dqn = _mod("dqn")
    mem = dqn.ReplayMemories(1, 2, 3, 4, "cpu")
    seq = iter([torch.tensor([[2, 0]]), torch.tensor([[1, 1]]), torch.tensor([[0, 2]]), torch.tensor([[1, 0]])])
    for t in range(5):
        s = torch.full((1, 2, 4), t, dtype=torch.int8)
        mem.push(s, s[..., 0], s[..., 0].float(), s, lambda: next(seq))
    # cap 3: pushes 0, 1 fill slots 0, 1 and push 1 (nextFreeIndex 2 == cap - 1) also replaces [2, 0];
    # pushes 2, 3, 4 replace by the draws only
    assert mem.next_free == 2
    assert mem.actions[0, :, :].tolist() == [[3, 4, 1], [4, 2, 3]]


def test_epsilon_schedule():
    dqn = _mod("dqn")
    hp = dqn.DQNHyper()
    assert dqn.epsilon(hp, 0) == pytest.approx(0.9)
    assert dqn.epsilon(hp, 500) == pytest.approx(0.05 + 0.85 * math.exp(-1))


def _compact(E, N, C, O, seed):
    g = torch.Generator().manual_seed(seed)
    D = 3 + 2 * O
    stride = (D + 3) // 4 * 4
    owners = torch.randint(0, N + 1, (E, C), generator=g).to(torch.int8)
    rows = torch.zeros((E, C, stride), dtype=torch.int8)
    rows[..., 0] = 1
    rows[..., 1:3] = torch.randint(1, 12, (E, C, 2), generator=g).to(torch.int8)
    rows[..., 3:D] = torch.randint(-2, 12, (E, C, D - 3), generator=g).to(torch.int8)
    return rows, owners, D


def test_structured_layer1_equals_dense_on_cpu():
    bdqn = _mod("bdqn")
    E, N, C, O = 6, 5, 4, 15
    rows, owners, D = _compact(E, N, C, O, 1)
    torch.manual_seed(0)
    net = bdqn.BranchingQ(C * D, C, O + 1)
    foreign = torch.tensor([0, -1, -1] + [-2] * (2 * O), dtype=torch.float32)
    x = torch.zeros((E * N, C * D))
    for e in range(E):
        for a in range(N):
            for c in range(C):
                x[e * N + a, c * D:(c + 1) * D] = rows[e, c, :D].float() if owners[e, c] == a + 1 else foreign
    from oracle.bdqn_ref import layer1_compact_reference
    with torch.no_grad():
        h_c = layer1_compact_reference(net.w1, net.b1, rows, owners, N, D)
        q_c = net.head(h_c)
        q_d = net(x)
    assert torch.allclose(q_c, q_d, rtol=1e-5, atol=1e-4)


def test_branching_update_matches_reference_on_cpu():
    bdqn = _mod("bdqn")

    class _CpuRole(bdqn.BranchingRole):  # torch Adam instead of the HIP Adam (CPU)
        def __init__(self, *a):
            self.q = bdqn.BranchingQ(*a[:3])
            self.target = bdqn.BranchingQ(*a[:3])
            self.target.load_state_dict(self.q.state_dict())
            self.cfg = a[3]
            self.opt = torch.optim.Adam(self.q.parameters(), lr=a[3].lr)
            self.update_counter = 0
            self.graph = False  # eager update (the HIP-graph capture needs a GPU)

    torch.manual_seed(2)
    obs, ac, n, B = 12, 3, 7, 32
    role = _CpuRole(obs, ac, n, bdqn.BDQNConfig())
    ref_q, ref_t = RefBranchingQNetwork(obs, ac, n), RefBranchingQNetwork(obs, ac, n)
    ref_q.load_stacked({k: getattr(role.q, k).detach() for k in bdqn.KEYS})
    ref_t.load_stacked({k: getattr(role.target, k).detach() for k in bdqn.KEYS})
    adam = torch.optim.Adam(ref_q.parameters(), lr=1e-4)
    g = torch.Generator().manual_seed(3)
    for _ in range(3):
        s, s1 = torch.randn((B, obs), generator=g), torch.randn((B, obs), generator=g)
        a = torch.randint(0, n, (B, ac), generator=g)
        r, m = torch.randn((B,), generator=g), (torch.rand((B,), generator=g) > 0.2).float()
        l1 = role.update(s, a, r, s1, m)
        l2 = update_policy_reference(ref_q, ref_t, adam, s, a, r, s1, m)
        assert abs(float(l1) - float(l2)) <= 1e-5 * max(1.0, abs(float(l2)))
    want = ref_q.stacked()
    for k in bdqn.KEYS:
        assert torch.allclose(getattr(role.q, k).detach(), want[k].detach(), rtol=1e-5, atol=1e-7), k


def test_episode_values_from_accumulators():
    abi = _mod("abi")
    mx = _mod("metrics")
    cfg = abi.make_config(2, 2, 2, [3, 10], [6, 3], [0.8, 0.2], fix_prices=[2, 7], episode_length=10)
    m = np.zeros(2, dtype=abi.metrics_dtype())
    m[0]["acceptor_reward"] = 40
    m[0]["offer_reward"] = 12
    m[0]["auctioneer_reward"] = 7
    m[0]["termination_revenue"] = 20
    m[0]["quality_sum"] = 3.0
    m[0]["quality_rounds"] = 2
    m[0]["acception_amount"] = 5
    m[0]["rounds"] = 10
    m[0]["price_sum"][1] = 21
    m[0]["price_count"][1] = 3
    m[0]["dwell_sum"][0] = 12
    m[0]["dwell_count"][0] = 2
    m[0]["agent_reward"][:2] = [15, 25]
    v = mx.episode_values(m, cfg, 10, 2, 2, 2)
    d = v[0]
    assert d["acceptorRew"] == pytest.approx(1.0) and d["coreChooserRew"] == pytest.approx(0.3)
    assert d["prices"] == [None, 7.0] and d["dwellTimes"] == [1.0, None]
    assert d["auctioneerRew"] == 0.7 and d["acceptionQuality"] == 1.5 and d["acceptionAmount"] == 0.5
    assert d["terminationRevenues"] == 0.5 and list(d["agentRew"]) == [1.5, 2.5]
    assert v[1]["acceptionQuality"] is None and v[1]["prices"] == [None, None]
    args = mx.args_dict([v], cfg, params=dict(episodeLength=10))
    assert args["acceptorRew"][0] == pytest.approx(0.5) and args["prices"][0] == [None, 7.0]
    assert float(args["meanJob"]) == pytest.approx((0.5 + 10 / 3) / 2)


def test_save_args_dict_picks_first_free_index(tmp_path):
    """trainPPO.py:245-251: data{i}.pkl with the first i whose file does not exist."""
    import pickle
    mx = _mod("metrics")
    paths = [mx.save_args_dict({"acceptorRew": [i]}, directory=str(tmp_path)) for i in range(3)]
    assert [p.rsplit("/", 1)[1] for p in paths] == ["data0.pkl", "data1.pkl", "data2.pkl"]
    with open(paths[2], "rb") as f:  # written by this test
        assert pickle.load(f) == {"acceptorRew": [2]}
