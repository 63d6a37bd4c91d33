"""Torch fp32 restatement of the reference's DQN unit and its optimisation step (CPU).

TEST INFRASTRUCTURE ONLY: checks marl-scheduling_amd/dqn.py + the ms_dqn_* kernels.
Follows (paths relative to /root/reference/src):
  DQNEntity            DQNmodules.py:34-76  nn.Sequential(Linear(D, 16), Tanh, Linear(16, A)),
                                            selectAction = argmax of Q unless epsilon explores
  optimize_model       DQNmodules.py:97-154 SmoothL1(Q(s)[a], r + GAMMA * max Q_target(s')),
                                            grads clamped to [-1, 1], Adam (torch defaults)
"""
from __future__ import annotations

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
