"""Torch fp32 restatement of the reference's Branching DQN (BranchingDQNModules.py) — TEST INFRASTRUCTURE ONLY.

BranchingQNetwork (BranchingDQNModules.py:75-101) with its ModuleList of advantage heads, and
BranchingDQN.update_policy (:125-164) on an already drawn batch; checks marl-scheduling_amd/bdqn.py.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class RefBranchingQNetwork(nn.Module):
    def __init__(self, obs, ac_dim, n):
        super().__init__()
        self.ac_dim = ac_dim
        self.n = n
        self.model = nn.Sequential(nn.Linear(obs, 128), nn.ReLU(), nn.Linear(128, 128), nn.ReLU())
        self.value_head = nn.Linear(128, 1)
        self.adv_heads = nn.ModuleList([nn.Linear(128, n) for i in range(ac_dim)])

    def forward(self, x):
        out = self.model(x)
        value = self.value_head(out)
        advs = torch.stack([l(out) for l in self.adv_heads], dim=1)
        q_val = value.unsqueeze(2) + advs - advs.mean(2, keepdim=True)
        return q_val

    def load_stacked(self, p):
        """Weights of the build's stacked layout: w1 b1 w2 b2 wv bv wa [ac_dim*n, 128] ba."""
        with torch.no_grad():
            self.model[0].weight.copy_(p["w1"])
            self.model[0].bias.copy_(p["b1"])
            self.model[2].weight.copy_(p["w2"])
            self.model[2].bias.copy_(p["b2"])
            self.value_head.weight.copy_(p["wv"])
            self.value_head.bias.copy_(p["bv"])
            for i, h in enumerate(self.adv_heads):
                h.weight.copy_(p["wa"][i * self.n:(i + 1) * self.n])
                h.bias.copy_(p["ba"][i * self.n:(i + 1) * self.n])

    def stacked(self):
        return dict(w1=self.model[0].weight, b1=self.model[0].bias, w2=self.model[2].weight, b2=self.model[2].bias,
                    wv=self.value_head.weight, bv=self.value_head.bias,
                    wa=torch.cat([h.weight for h in self.adv_heads]), ba=torch.cat([h.bias for h in self.adv_heads]))


def update_policy_reference(q, target, adam, states, actions, rewards, next_states, masks):
    """BranchingDQN.update_policy (BranchingDQNModules.py:127-159) after memory.sample."""
    actions = actions.long().reshape(states.shape[0], -1, 1)
    rewards = rewards.float().reshape(-1, 1)
    masks = masks.float().reshape(-1, 1)
    current_q_values = q(states).gather(2, actions).squeeze(-1)
    with torch.no_grad():
        argmax = torch.argmax(q(next_states), dim=2)
        max_next_q_vals = target(next_states).gather(2, argmax.unsqueeze(2)).squeeze(-1)
        max_next_q_vals = max_next_q_vals.mean(1, keepdim=True)
    expected_q_vals = rewards + max_next_q_vals * 0.99 * masks
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # the reference broadcasts [B, 1] against [B, ac_dim]
        loss = F.mse_loss(expected_q_vals, current_q_values)
    adam.zero_grad()
    loss.backward()
    for p in q.parameters():
        p.grad.data.clamp_(-1.0, 1.0)
    adam.step()
    return loss.detach()


def layer1_compact_reference(w1, b1, core_rows, core_owner, n_agents: int, d_acc: int):
    """The structured layer 1 of the aggregated acceptor rows in torch fp32 (the algebra
    ms_bdqn_layer1_compact implements): an agent's row is R_c on the cores it owns and the foreign
    row F elsewhere (Agent.py:167-212), so W1 x_a + b1 = (b1 + sum_c W1_c F) + sum_{c owned by a}
    W1_c (R_c - F). core_rows [E, C, stride] int8, core_owner [E, C] -> [E * N, 128]."""
    E, C, _ = core_rows.shape
    O = (d_acc - 3) // 2
    foreign = torch.tensor([0.0, -1.0, -1.0] + [-2.0] * (2 * O), device=core_rows.device)
    w1c = w1.view(w1.shape[0], C, d_acc)
    base = b1 + torch.einsum("jcd,d->j", w1c, foreign)
    dc = core_rows[:, :, :d_acc].float() - foreign
    part = torch.bmm(dc.transpose(0, 1), w1c.permute(1, 2, 0))             # [C, E, 128]
    h1 = base.expand(E * n_agents, w1.shape[0]).contiguous()
    own = core_owner.long()
    mask = own > 0
    rows = (torch.arange(E, device=own.device).unsqueeze(1) * n_agents + own - 1)[mask]
    return h1.index_add(0, rows, part.transpose(0, 1)[mask])
