"""Drop-in ``PPOmodules`` module (PPOmodules.py:9-72 names).

In this build the PPO objects of all units of one type are grouped inside the
env (``SchedulingEnvironment.PPOSchedulingEnv``): acting runs on the HIP act
kernels and updates on the fused gradient kernel. This module keeps the
reference's public building blocks for code that imports them:

* ``ExperienceBuffer``;
* ``ActorCritic`` (same layers and ``act``/``evaluate`` semantics);
* ``unit_actor_critic(env, kind, index)``, which returns the current weights of
  one unit as an ``ActorCritic``, e.g. to save or inspect a trained net.
"""
from __future__ import annotations

import math  # noqa: F401
from collections import deque  # noqa: F401

import torch
import torch.nn as nn
from torch.distributions import Categorical

from marlsched_dropin import ppo

__all__ = ["ExperienceBuffer", "ActorCritic", "unit_actor_critic", "torch", "nn", "Categorical"]


class ExperienceBuffer:
    """Per-unit rollout lists (PPOmodules.py:9-22)."""

    def __init__(self):
        self.actions, self.states, self.logprobs, self.rewards = [], [], [], []

    def clear(self):
        for lst in (self.actions, self.states, self.logprobs, self.rewards):
            del lst[:]


class ActorCritic(nn.Module):
    """Linear-Tanh-Linear-Tanh-Linear-Softmax actor and Linear-Tanh-Linear-Tanh-Linear critic
    (PPOmodules.py:25-72); hidden width numberOfNeurons."""

    def __init__(self, amountInputChannels, numberOfActions, numberOfNeurons):
        super().__init__()
        H = numberOfNeurons
        self.actor = nn.Sequential(nn.Linear(amountInputChannels, H), nn.Tanh(), nn.Linear(H, H), nn.Tanh(),
                                   nn.Linear(H, numberOfActions), nn.Softmax(dim=-1))
        self.critic = nn.Sequential(nn.Linear(amountInputChannels, H), nn.Tanh(), nn.Linear(H, H), nn.Tanh(),
                                    nn.Linear(H, 1))

    def forward(self):
        raise NotImplementedError

    def act(self, state):
        dist = Categorical(self.actor(state))
        action = dist.sample()
        return action.detach(), dist.log_prob(action).detach()

    def evaluate(self, state, action):
        dist = Categorical(self.actor(state))
        return dist.log_prob(action), self.critic(state).squeeze(), dist.entropy()


_LAYER_KEYS = [("actor.0", "w1", "b1"), ("actor.2", "w2", "b2"), ("actor.4", "w3", "b3"),
               ("critic.0", "cw1", "cb1"), ("critic.2", "cw2", "cb2"), ("critic.4", "cw3", "cb3")]


def unit_actor_critic(env, kind: str, index: int, old: bool = False) -> ActorCritic:
    """Group ``index`` of unit type ``kind`` ("acc", "off" or "price") of a drop-in PPO env, as an
    ActorCritic on the CPU (policy, or policy_old with old=True)."""
    grp = env._units[kind].group
    net = grp.policy_old if old else grp.policy
    ac = ActorCritic(net.D, net.A, net.H)
    sd = {}
    for prefix, w, b in _LAYER_KEYS:
        sd[prefix + ".weight"] = getattr(net, w)[index].detach().cpu()
        sd[prefix + ".bias"] = getattr(net, b)[index].detach().cpu()
    ac.load_state_dict(sd)
    return ac


assert ppo.ACTOR_KEYS == ("w1", "b1", "w2", "b2", "w3", "b3")
