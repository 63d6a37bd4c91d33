"""Torch-fp32 CPU restatement of the reference PPO (PPOmodules.py:9-174).

TEST INFRASTRUCTURE ONLY: the checker for the product's batched PPO (act
kernel, returns kernel, grouped update). One ``RefPPO`` is one unit's
``PPO`` object: an ActorCritic built with nn.Linear defaults (policy, then
policy_old), Adam with actor/critic parameter groups, Monte-Carlo returns in
Python floats, K epochs of the clipped objective. Parity status: pinned to the
formulas of PPOmodules.py and torch's own Categorical/Adam (no reference
outputs exist to pin against).
"""
from __future__ import annotations

from collections import deque

import torch
import torch.nn as nn
from torch.distributions import Categorical


class RefActorCritic(nn.Module):  # PPOmodules.py:25-72
    def __init__(self, d, a, h=16):
        super().__init__()
        self.actor = nn.Sequential(nn.Linear(d, h), nn.Tanh(), nn.Linear(h, h), nn.Tanh(), nn.Linear(h, a),
                                   nn.Softmax(dim=-1))
        self.critic = nn.Sequential(nn.Linear(d, h), nn.Tanh(), nn.Linear(h, h), nn.Tanh(), nn.Linear(h, 1))

    def evaluate(self, state, action):
        probs = self.actor(state)
        dist = Categorical(probs)
        return dist.log_prob(action), self.critic(state).squeeze(), dist.entropy()

    def flat(self):
        a, c = self.actor, self.critic
        return dict(w1=a[0].weight, b1=a[0].bias, w2=a[2].weight, b2=a[2].bias, w3=a[4].weight, b3=a[4].bias,
                    cw1=c[0].weight, cb1=c[0].bias, cw2=c[2].weight, cb2=c[2].bias, cw3=c[4].weight, cb3=c[4].bias)


class RefPPO:
    def __init__(self, d, a, lr_actor, lr_critic, gamma, eps_clip, k_epochs, h=16):
        self.gamma, self.eps_clip, self.K = gamma, eps_clip, k_epochs
        self.policy = RefActorCritic(d, a, h)
        self.optimizer = torch.optim.Adam([
            {"params": self.policy.actor.parameters(), "lr": lr_actor},
            {"params": self.policy.critic.parameters(), "lr": lr_critic},
        ], foreach=False)
        self.policy_old = RefActorCritic(d, a, h)
        self.policy_old.load_state_dict(self.policy.state_dict())
        self.mse = nn.MSELoss()

    def returns(self, rewards):
        """Monte-Carlo returns (PPOmodules.py:128-137): Python floats, then f32, then normalised."""
        out = deque([])
        g = 0
        for r in reversed(list(rewards)):
            g = r + (self.gamma * g)
            out.appendleft(g)
        t = torch.tensor(out, dtype=torch.float32)
        return (t - t.mean()) / (t.std() + 1e-7)

    def epoch(self, states, actions, old_logprobs, rewards_norm):
        """One K-epoch step of PPOmodules.py:144-168: the clipped-surrogate loss, its gradient, the Adam
        step. Returns (mean loss, {name: the gradient before the step})."""
        logprobs, values, entropy = self.policy.evaluate(states, actions)
        ratios = torch.exp(logprobs - old_logprobs.detach())
        adv = rewards_norm - values.detach()
        s1 = ratios * adv
        s2 = torch.clamp(ratios, 1 - self.eps_clip, 1 + self.eps_clip) * adv
        loss = -torch.min(s1, s2) + 0.5 * self.mse(values, rewards_norm) - 0.01 * entropy
        self.optimizer.zero_grad()
        loss.mean().backward()
        grads = {k: v.grad.detach().clone() for k, v in self.policy.flat().items()}
        self.optimizer.step()
        return float(loss.mean().detach()), grads

    def update(self, states, actions, old_logprobs, rewards_norm):
        """PPOmodules.py:144-171 on given tensors; returns the per-epoch mean losses."""
        losses = [self.epoch(states, actions, old_logprobs, rewards_norm)[0] for _ in range(self.K)]
        self.policy_old.load_state_dict(self.policy.state_dict())
        return losses


def act_reference(flat: dict, obs: torch.Tensor, u: torch.Tensor):
    """ActorCritic.act with an inverse-CDF sample at uniform u (rows of obs, float32)."""
    h = torch.tanh(obs @ flat["w1"].T + flat["b1"])
    h = torch.tanh(h @ flat["w2"].T + flat["b2"])
    probs = torch.softmax(h @ flat["w3"].T + flat["b3"], dim=-1)
    dist = Categorical(probs)
    cdf = torch.cumsum(dist.probs, dim=-1)
    a = (u.unsqueeze(-1) >= cdf).sum(-1).clamp(max=probs.shape[-1] - 1)
    return a, dist.log_prob(a), dist.probs


def grad_abs_bound(policy: RefActorCritic, states, actions, old_logprobs, rewards_norm, eps_clip: float):
    """The per-element scale a summed gradient's rounding error is measured against: for every Linear layer
    y = x W^T + b of the actor and the critic, sum over rows of |dL/dy_r| (x) |x_r| (weights) and of |dL/dy_r|
    (biases), in the precision of `policy` (use float64). The gradient of PPOmodules.py:144-168's mean loss is
    sum_r dL/dy_r (x) x_r: when its rows cancel, the sum is far smaller than these terms, and an f32 sum's error
    is a fraction of the terms (~ log2(rows) * 2^-24 for a blocked sum), not of the sum. TEST INFRASTRUCTURE."""
    seen = {}

    def hook(name):
        def f(mod, inp, out):
            out.retain_grad()
            seen[name] = (inp[0].detach(), out)
        return f

    layers = dict(w1=policy.actor[0], w2=policy.actor[2], w3=policy.actor[4], cw1=policy.critic[0],
                  cw2=policy.critic[2], cw3=policy.critic[4])
    handles = [lin.register_forward_hook(hook(k)) for k, lin in layers.items()]
    try:
        logprobs, values, entropy = policy.evaluate(states, actions)
        ratios = torch.exp(logprobs - old_logprobs.detach())
        adv = rewards_norm - values.detach()
        s1 = ratios * adv
        s2 = torch.clamp(ratios, 1 - eps_clip, 1 + eps_clip) * adv
        loss = -torch.min(s1, s2) + 0.5 * nn.MSELoss()(values, rewards_norm) - 0.01 * entropy
        policy.zero_grad()
        loss.mean().backward()
    finally:
        for h in handles:
            h.remove()
    out = {}
    for k, (x, y) in seen.items():
        d = y.grad.detach().abs()
        out[k] = d.T @ x.abs()
        out[k.replace("w", "b")] = d.sum(0)
    policy.zero_grad()
    return out
