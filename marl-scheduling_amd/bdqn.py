"""Branching DQN (BranchingDQNModules.py) for the scheduling agents, BASELINE cfg5 (32 agents x 32 cores).

The reference module is a stand-alone template (BranchingDQNModules.py:167-208 runs it on an
undefined gym ``env``): a dueling BranchingQNetwork (trunk Linear(obs,128)-ReLU-Linear(128,128)-ReLU,
value head, one advantage head of n actions per action dimension, q = value + adv - mean(adv),
:75-101), epsilon-greedy ``get_action`` (:117-123), an ExperienceReplayMemory (:43-72) and
``update_policy`` (:125-164: double-DQN target averaged over the branches, MSE loss, every gradient
element clamped to [-1, 1], Adam lr 1e-4, target sync every 1000 updates). This build wires it to
the scheduling env per agent, with three roles whose branches are the agent's divided decisions:

  acceptor  obs = the agent's C acceptor rows (AggregatedAgent's acceptor row, Agent.py:82-124,
            C * D_acc values), C branches of O + 1 actions (offer index, O = reject);
  offerer   obs = the cores' (prio, rem) + the agent's slots' (prio, rem) (Agent.py:126-134),
            L branches of C + 1 actions (core index, C = no offer);
  price     (free prices) the offerer's obs, L branches of max(priorities) + 1 prices;

one net per role shared by all agents (the observations are agent-relative), rewards the agent's
aggregated acceptor / offer rewards (getAggregatedFixedPricesReward, Reward.py:92-143) and the sum
of its slots' priceChooser rewards.

MI355X design. At cfg5 an agent's acceptor observation is 6240 bytes, 200 KB per env-round: a
replay memory of materialised observations would hold ~40 frames of 8192 replicas in 288 GB.
Instead every frame stores the env kernel's compact observations (ms_obs_out.core_rows /
core_owner: the C owner rows, 6.3 KB per env) and the slot pairs, and the acceptor rows are
regenerated from them: for the minibatch by ``ms_regen_agent_rows``; for acting, where all N
agents of all replicas need layer 1, by its algebra. An agent's row is the owner row R_c where it
owns core c and the constant foreign row F elsewhere, so
    W1 x_a + b1 = (b1 + sum_c W1_c F) + sum_{c owned by a} W1_c (R_c - F),
one [E, D] x [D, 128] GEMM per core (torch.bmm over cores) scattered to the owners: C GEMVs per
replica instead of N dense [C*D]-wide ones (32x fewer flops at cfg5). The trunk and heads are
plain library GEMMs (hipBLASLt through torch, fp32 like the reference).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F_

from . import abi
from .ppo import HipAdam

KEYS = ("w1", "b1", "w2", "b2", "wv", "bv", "wa", "ba")


class BranchingQ(nn.Module):
    """BranchingQNetwork (BranchingDQNModules.py:75-101) with the advantage heads stacked into one
    [ac_dim * n, 128] matrix (head i = rows i*n .. i*n+n-1); initialised in the reference's order."""

    def __init__(self, obs: int, ac_dim: int, n: int):
        super().__init__()
        self.obs, self.ac_dim, self.n = obs, ac_dim, n
        l1, l2 = nn.Linear(obs, 128), nn.Linear(128, 128)
        v = nn.Linear(128, 1)
        heads = [nn.Linear(128, n) for _ in range(ac_dim)]
        self.w1, self.b1 = nn.Parameter(l1.weight.detach().clone()), nn.Parameter(l1.bias.detach().clone())
        self.w2, self.b2 = nn.Parameter(l2.weight.detach().clone()), nn.Parameter(l2.bias.detach().clone())
        self.wv, self.bv = nn.Parameter(v.weight.detach().clone()), nn.Parameter(v.bias.detach().clone())
        self.wa = nn.Parameter(torch.cat([h.weight.detach() for h in heads]).clone())
        self.ba = nn.Parameter(torch.cat([h.bias.detach() for h in heads]).clone())

    def head(self, h1_pre):
        """ReLU(h1_pre) -> Linear-ReLU -> value + advantages - mean (BranchingDQNModules.py:88-101)."""
        out = torch.relu(F_.linear(torch.relu(h1_pre), self.w2, self.b2))
        value = F_.linear(out, self.wv, self.bv)
        advs = F_.linear(out, self.wa, self.ba).view(-1, self.ac_dim, self.n)
        return value.unsqueeze(2) + advs - advs.mean(2, keepdim=True)

    def greedy(self, h1_pre):
        """get_action's argmax (BranchingDQNModules.py:117-123) without materialising q: value and the
        advantage mean are constant along a branch, so argmax q = argmax advantage (torch.argmax's
        first-maximum rule may differ from q's only on exact float ties)."""
        out = torch.relu(F_.linear(torch.relu(h1_pre), self.w2, self.b2))
        return torch.argmax(F_.linear(out, self.wa, self.ba).view(-1, self.ac_dim, self.n), dim=2)

    def forward(self, x):
        """x [B, obs] float -> q [B, ac_dim, n]."""
        return self.head(F_.linear(x, self.w1, self.b1))

    def layer1_compact(self, core_rows, core_owner, n_agents: int, d_acc: int):
        """Layer-1 pre-activations of every agent's acceptor row from the compact observations (module doc):
        core_rows [E, C, stride] int8, core_owner [E, C] int8 -> [E * N, 128] (row e * N + a)."""
        E, C, _ = core_rows.shape
        O = (d_acc - 3) // 2
        foreign = torch.tensor([0.0, -1.0, -1.0] + [-2.0] * (2 * O), device=core_rows.device)
        w1c = self.w1.view(128, C, d_acc)                                     # W1_c = w1c[:, c, :]
        base = self.b1 + torch.einsum("jcd,d->j", w1c, foreign)               # b1 + sum_c W1_c F
        dc = core_rows[:, :, :d_acc].float() - foreign                        # R_c - F  [E, C, D]
        part = torch.bmm(dc.transpose(0, 1), w1c.permute(1, 2, 0))             # [C, E, 128]
        h1 = base.expand(E * n_agents, 128).contiguous()
        own = core_owner.long()                                               # [E, C], 0 = auctioneer
        mask = own > 0
        rows = (torch.arange(E, device=own.device).unsqueeze(1) * n_agents + own - 1)[mask]
        h1 = h1.index_add(0, rows, part.transpose(0, 1)[mask])
        return h1

    def forward_compact(self, core_rows, core_owner, n_agents: int, d_acc: int):
        """q [E * N, C, n] of every agent from the compact observations (layer1_compact + head)."""
        return self.head(self.layer1_compact(core_rows, core_owner, n_agents, d_acc))


@dataclass
class BDQNConfig:
    """AgentConfig (BranchingDQNModules.py:10-40); memory and learning start in frames of E x N
    transitions (one frame = one round of every replica's agents)."""
    epsilon_start: float = 1.0
    epsilon_final: float = 0.01
    epsilon_decay: float = 8000
    gamma: float = 0.99
    lr: float = 1e-4
    target_net_update_freq: int = 1000
    memory_frames: int = 16
    batch_size: int = 128
    learning_starts: int = 4
    grad_clip: float = 1.0

    def epsilon_by_frame(self, i):
        return self.epsilon_final + (self.epsilon_start - self.epsilon_final) * math.exp(-1.0 * i / self.epsilon_decay)


class BranchingRole:
    """BranchingDQN (BranchingDQNModules.py:104-164) of one role: online / target nets, Adam, counter."""

    def __init__(self, obs: int, ac_dim: int, n: int, cfg: BDQNConfig, device):
        self.q = BranchingQ(obs, ac_dim, n).to(device)
        self.target = BranchingQ(obs, ac_dim, n).to(device)  # its own init draw, then overwritten (:110-112)
        self.target.load_state_dict(self.q.state_dict())
        self.target.requires_grad_(False)
        self.cfg = cfg
        self.opt = HipAdam([dict(params=list(self.q.parameters()), lr=cfg.lr)])
        self.update_counter = 0

    def update(self, states, actions, rewards, next_states, masks):
        """update_policy (BranchingDQNModules.py:125-164) on a drawn batch: states / next_states [B, obs]
        float, actions [B, ac_dim] long, rewards / masks [B]. Returns the loss."""
        current = self.q(states).gather(2, actions.unsqueeze(2)).squeeze(-1)
        with torch.no_grad():
            argmax = torch.argmax(self.q(next_states), dim=2)
            max_next = self.target(next_states).gather(2, argmax.unsqueeze(2)).squeeze(-1).mean(1, keepdim=True)
        expected = rewards.view(-1, 1) + max_next * self.cfg.gamma * masks.view(-1, 1)
        loss = ((expected - current) ** 2).mean()  # F.mse_loss(expected, current) broadcast over branches
        self.opt.zero_grad()
        loss.backward()
        for p in self.q.parameters():
            p.grad.data.clamp_(-self.cfg.grad_clip, self.cfg.grad_clip)
        self.opt.step()
        self.update_counter += 1
        if self.update_counter % self.cfg.target_net_update_freq == 0:
            self.update_counter = 0
            self.target.load_state_dict(self.q.state_dict())
        return loss.detach()


class BDQNTrainer:
    """The BranchingDQN loop (BranchingDQNModules.py:175-208) over E replicas of the scheduling env,
    every agent an actor of the shared role nets; the replay memory keeps compact frames."""

    def __init__(self, cfg: abi.MsConfig, n_envs: int, bcfg: BDQNConfig | None = None, seed: int = 0, device=None,
                 episode_length: int | None = None):
        from .env import BatchedEnv
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        torch.cuda.set_device(self.device)
        if episode_length is not None:
            cfg = abi.MsConfig.from_buffer_copy(cfg)
            cfg.episode_length = int(episode_length)
        self.cfg, self.E, self.b = cfg, int(n_envs), bcfg or BDQNConfig()
        self.env = BatchedEnv(cfg, self.E, seed=seed, device=self.device)
        s = self.env.shape
        N, C, L, O = s.n_agents, s.n_cores, s.collection_length, s.max_offers
        self.N, self.C, self.L, self.O = N, C, L, O
        self.free = bool(cfg.free_prices)
        self.d_acc, self.stride = s.acc_obs_dim, s.acc_obs_stride
        dims = self.env.aggregated_dims()
        self.d_off, self.ld_off = dims["offer"]
        self.ld_acc = dims["acceptor"][1]
        torch.manual_seed(seed)
        dev = self.device
        self.roles = dict(acc=BranchingRole(C * s.acc_obs_dim, C, O + 1, self.b, dev),
                          off=BranchingRole(self.d_off, L, C + 1, self.b, dev))
        if self.free:
            self.roles["price"] = BranchingRole(self.d_off, L, s.price_actions, self.b, dev)
        # compact replay ring: states of frames 0..F (slot F + 1 holds the next state of the newest frame)
        Fm = self.b.memory_frames
        self.n_slots = Fm + 1
        E = self.E
        self.core_rows = torch.zeros((self.n_slots, E, C, self.stride), dtype=torch.int8, device=dev)
        self.core_owner = torch.zeros((self.n_slots, E, C), dtype=torch.int8, device=dev)
        self.slot_pairs = torch.zeros((self.n_slots, E, N, L, 2), dtype=torch.int8, device=dev)
        self.act = {k: torch.zeros((self.n_slots, E, N, r.q.ac_dim), dtype=torch.int8, device=dev)
                    for k, r in self.roles.items()}
        self.rew = {k: torch.zeros((self.n_slots, E, N), dtype=torch.float32, device=dev) for k in self.roles}
        self.mask = torch.ones(self.n_slots, dtype=torch.float32, device=dev)
        self.off_rows = torch.zeros((E, N, L, s.off_obs_stride), dtype=torch.int8, device=dev)
        self.rbuf = self.env.reward_buffers(aggregated=True)
        self.rbuf["price"] = torch.zeros((E, N, L), dtype=torch.float32, device=dev) if self.free else None
        self.head = 0      # ring slot of the current state
        self.stored = 0    # frames stored (<= memory_frames)
        self.frame = 0
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed + 17)
        self._agent_idx = torch.arange(N, dtype=torch.int32, device=dev).repeat(E)
        self._observe_into(self.head, reset=True)
        self._store_slot_pairs(self.head)
        self.last_losses = {}

    def _observe_into(self, slot, reset=False):
        obs = dict(core_rows=self.core_rows[slot], core_owner=self.core_owner[slot], offer=self.off_rows)
        if reset:
            self.env.reset(obs)
        return obs

    def _store_slot_pairs(self, slot):
        self.slot_pairs[slot].copy_(self.off_rows[..., 2 * self.C:2 * self.C + 2])

    def _offer_rows(self, slot):
        """The aggregated offer rows of every (replica, agent) of ring slot `slot` (ms_regen_agent_rows)."""
        E, N = self.E, self.N
        frame = (torch.arange(E, device=self.device, dtype=torch.int64) + slot * E).repeat_interleave(N)
        _, off = self.env.regen_agent_rows(self.core_rows.view(-1, self.C, self.stride),
                                           self.core_owner.view(-1, self.C), self.slot_pairs.view(-1, N, self.L, 2),
                                           frame, self._agent_idx,
                                           offer=torch.empty((E * N, self.ld_off), dtype=torch.int8,
                                                             device=self.device))
        return off[:, : self.d_off].float()

    @torch.no_grad()
    def _actions(self, slot, eps):
        """get_action (BranchingDQNModules.py:117-123) of every agent, epsilon-greedy per agent (:181-186)."""
        E, N = self.E, self.N
        qa = self.roles["acc"].q
        h1 = dict(acc=qa.layer1_compact(self.core_rows[slot], self.core_owner[slot], N, self.d_acc))
        x_off = self._offer_rows(slot)
        for k in ("off", "price"):
            if k in self.roles:
                q = self.roles[k].q
                h1[k] = F_.linear(x_off, q.w1, q.b1)
        explore = torch.rand((E * N,), generator=self.gen, device=self.device) <= eps
        out = {}
        for k, h in h1.items():
            q = self.roles[k].q
            greedy = q.greedy(h)
            rnd = torch.randint(0, q.n, greedy.shape, generator=self.gen, device=self.device)
            out[k] = torch.where(explore.unsqueeze(1), rnd, greedy).to(torch.int8).view(E, N, -1)
        return out

    def step(self):
        """One frame: act, env.step, store the transition, learn (BranchingDQNModules.py:179-208)."""
        E, N, C, L = self.E, self.N, self.C, self.L
        b = self.b
        cur = self.head
        nxt = (cur + 1) % self.n_slots
        eps = b.epsilon_by_frame(self.frame)
        acts = self._actions(cur, eps)
        for k, a in acts.items():
            self.act[k][cur].copy_(a)
        obs = self._observe_into(nxt)
        price = acts["price"].contiguous() if self.free else None
        rew = dict(self.rbuf)
        self.env.step(acts["acc"].contiguous(), acts["off"].contiguous(), price, obs=obs, rewards=rew)
        self._store_slot_pairs(nxt)
        done = self.env.round % self.cfg.episode_length == 0
        self.rew["acc"][cur].copy_(rew["aggregated_acceptor"].float())
        self.rew["off"][cur].copy_(rew["aggregated_offer"].float())
        if self.free:
            self.rew["price"][cur].copy_(rew["price"].sum(2))
        self.mask[cur] = 0.0 if done else 1.0
        self.head = nxt
        self.stored = min(self.stored + 1, self.b.memory_frames)
        self.frame += 1
        if self.frame > b.learning_starts:
            self._learn()
        return done

    def _sample(self):
        """batch_size transitions uniformly from the stored frames' E x N transitions: (ring slot, env, agent)."""
        E, N, B = self.E, self.N, self.b.batch_size
        j = torch.randint(0, self.stored * E * N, (B,), generator=self.gen, device=self.device)
        age = j // (E * N)                                      # 0 = newest stored frame
        slot = (self.head - 1 - age) % self.n_slots
        e = (j // N) % E
        a = (j % N).to(torch.int32)
        return slot, e, a

    def _learn(self):
        slot, e, a = self._sample()
        nslot = (slot + 1) % self.n_slots
        rec, nrec = slot * self.E + e, nslot * self.E + e
        cr = self.core_rows.view(-1, self.C, self.stride)
        co = self.core_owner.view(-1, self.C)
        sp = self.slot_pairs.view(-1, self.N, self.L, 2)
        acc_s, off_s = self.env.regen_agent_rows(cr, co, sp, rec, a)
        acc_n, off_n = self.env.regen_agent_rows(cr, co, sp, nrec, a)
        xs = dict(acc=(acc_s[:, : self.C * self.d_acc].float(), acc_n[:, : self.C * self.d_acc].float()),
                  off=(off_s[:, : self.d_off].float(), off_n[:, : self.d_off].float()))
        xs["price"] = xs["off"]
        masks = self.mask[slot]
        losses = {}
        for k, role in self.roles.items():
            s, s1 = xs[k]
            acts = self.act[k][slot, e, a.long()].long()
            r = self.rew[k][slot, e, a.long()]
            losses[k] = role.update(s, acts, r, s1, masks)
        self.last_losses = losses

    def flags(self) -> int:
        return self.env.flags()
