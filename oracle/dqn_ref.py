"""Torch fp32 restatement of the reference's DQN unit and its optimisation step (CPU).

TEST INFRASTRUCTURE ONLY: checks marl-scheduling_amd/dqn.py + the ms_dqn_* kernels.
Follows (paths relative to /root/reference/src):
  DQNEntity            DQNmodules.py:34-76  nn.Sequential(Linear(D, 16), Tanh, Linear(16, A)),
                                            selectAction = argmax of Q unless epsilon explores
  optimize_model       DQNmodules.py:97-154 SmoothL1(Q(s)[a], r + GAMMA * max Q_target(s')),
                                            grads clamped to [-1, 1], Adam (torch defaults)
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn


class RefDQNEntity(nn.Module):
    """DQNEntity's model (DQNmodules.py:41-46) with given weights."""

    def __init__(self, w1, b1, w2, b2):
        super().__init__()
        D, A = w1.shape[1], w2.shape[0]
        self.model = nn.Sequential(nn.Linear(D, 16), nn.Tanh(), nn.Linear(16, A))
        with torch.no_grad():
            self.model[0].weight.copy_(w1)
            self.model[0].bias.copy_(b1)
            self.model[2].weight.copy_(w2)
            self.model[2].bias.copy_(b2)

    def forward(self, x):  # DQNmodules.py:52-54
        return self.model(x.float())

    def params(self):
        m = self.model
        return [m[0].weight, m[0].bias, m[2].weight, m[2].bias]


def optimize_model_reference(policy: RefDQNEntity, target: RefDQNEntity, optimizer, states, actions, next_states,
                             rewards, gamma: float, clip: bool = True):
    """One optimize_model call (DQNmodules.py:119-154) on an already drawn batch:
    states / next_states [B, D] int64, actions [B] (int or float), rewards [B] int64 or float.
    Returns the loss; the step leaves the (clamped) gradients in policy's .grad."""
    state_batch = states
    action_batch = actions.reshape(-1, 1)
    reward_batch = rewards.reshape(-1, 1)
    state_action_values = policy(state_batch).gather(1, action_batch.long())
    next_state_values = target(next_states).max(1)[0].detach()
    expected_state_action_values = (next_state_values * gamma) + reward_batch.squeeze(1)
    criterion = nn.SmoothL1Loss()
    loss = criterion(state_action_values, expected_state_action_values.unsqueeze(1))
    optimizer.zero_grad()
    loss.backward()
    if clip:
        for param in policy.parameters():
            param.grad.data.clamp_(-1, 1)
    optimizer.step()
    return loss.detach()


class RefReplayMemory:
    """ReplayMemory (DQNmodules.py:13-31) drawing its replacement index from the given random.Random."""

    def __init__(self, capacity, rng):
        self.memory = [None] * capacity
        self.nextFreeIndex = 0
        self.capacity = capacity
        self.rng = rng

    def push(self, *args):
        if (self.nextFreeIndex + 1) < self.capacity:
            self.memory[self.nextFreeIndex] = args
            self.nextFreeIndex += 1
        if (self.nextFreeIndex + 1) == self.capacity:
            self.memory[self.rng.randint(0, (self.capacity - 1))] = args

    def sample(self, batch_size):  # np.random.choice(self.memory[:nextFreeIndex], batch_size)
        idx = np.random.choice(self.nextFreeIndex, batch_size)
        return [self.memory[i] for i in idx]


class RefDQNAgents:
    """DividedFixPriceDQNAgent (Agent.py:303-356) of every agent plus DQNSchedulingEnv's updates
    (SchedulingEnvironment.py:366-425), on the object-faithful world's random stream."""

    def __init__(self, world, dims, params):
        import copy
        self.w = world
        N, C, L = world.N, world.C, world.L
        self.p = params
        self.policy = {"acc": [], "off": []}
        for _ in range(N):  # Agent.py:306-309 construction order
            for _ in range(C):
                self.policy["acc"].append(nn.Sequential(nn.Linear(dims["acc"][0], 16), nn.Tanh(),
                                                        nn.Linear(16, dims["acc"][1])))
            for _ in range(L):
                self.policy["off"].append(nn.Sequential(nn.Linear(dims["off"][0], 16), nn.Tanh(),
                                                        nn.Linear(16, dims["off"][1])))
        self.target = copy.deepcopy(self.policy)
        self.opt = {k: [torch.optim.Adam(n.parameters()) for n in v] for k, v in self.policy.items()}
        cap = params["REPLAY_MEMORY_SIZE"]
        self.mem = {k: [RefReplayMemory(cap, world.rng) for _ in v] for k, v in self.policy.items()}
        self.n_actions = {k: dims[k][1] for k in dims}

    def _select(self, kind, u, obs_row):  # DQNEntity.selectAction (DQNmodules.py:56-70)
        p = self.p
        sample = self.w.rng.random()
        eps = p["RUN_END"] + (p["RUN_START"] - p["RUN_END"]) * math.exp(-1.0 * self.w.round / p["RUN_DECAY"])
        if sample > eps:
            with torch.no_grad():
                return self.policy[kind][u](torch.tensor(obs_row).float()).max(0)[1].item()
        return float(self.w.rng.randrange(self.n_actions[kind]))

    def get_actions(self, acc_obs, off_obs):
        N, C, L = self.w.N, self.w.C, self.w.L
        acc, off = [], []
        for a in range(N):  # getActions: offer nets, then acceptor nets (Agent.py:345-356)
            off.append([self._select("off", a * L + j, off_obs[a][j]) for j in range(L)])
            acc.append([self._select("acc", a * C + c, acc_obs[a][c]) for c in range(C)])
        return acc, off

    def update(self, kind, actions, rewards, old_obs, new_obs, gamma):
        """updateXMemoriesAndOptimize: per agent, per unit: push then optimize_model."""
        per = self.w.C if kind == "acc" else self.w.L
        losses = []
        for a in range(self.w.N):
            for j in range(per):
                u = a * per + j
                mem = self.mem[kind][u]
                mem.push(tuple(old_obs[a][j]), actions[a][j], tuple(new_obs[a][j]), np.asarray(rewards[a][j]))
                if mem.capacity < self.p["BATCH_SIZE"]:
                    continue
                tr = mem.sample(self.p["BATCH_SIZE"])
                states = torch.cat([torch.tensor(t[0]).unsqueeze(0) for t in tr])
                acts = torch.cat([torch.tensor(t[1]).unsqueeze(0).unsqueeze(0) for t in tr])
                nexts = torch.cat([torch.tensor(t[2]).unsqueeze(0) for t in tr])
                rews = torch.cat([torch.tensor(t[3]).unsqueeze(0) for t in tr])
                pol = _Wrap(self.policy[kind][u])
                tgt = _Wrap(self.target[kind][u])
                losses.append(optimize_model_reference(pol, tgt, self.opt[kind][u], states, acts, nexts, rews, gamma))
        return losses

    def update_targets(self, agent):  # Agent.updateTargetNets (Agent.py:329-334)
        C, L = self.w.C, self.w.L
        for kind, per in (("acc", C), ("off", L)):
            for u in range(agent * per, (agent + 1) * per):
                self.target[kind][u].load_state_dict(self.policy[kind][u].state_dict())


class _Wrap(nn.Module):
    """DQNEntity.forward (x.float()) around a bare nn.Sequential."""

    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, x):
        return self.model(x.float())
