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
one [D, 128] product per (replica, core) added to its owner's row: C of them per replica instead
of N dense [C*D]-wide ones (32x fewer flops at cfg5), on the bf16 MFMA with exact products
(ms_bdqn_layer1_compact, bdqn_kernels.hip). Acting is one fused HIP kernel per role
(ms_bdqn_act; the acceptor role ms_bdqn_act_compact, which also adds the owned cores' layer-1 rows
itself): trunk, value head, every advantage head, the per-branch q = value + adv - mean and its
first argmax, and the epsilon-greedy pick, on the bf16 MFMA with both operands as three exact bf16
terms (six products: f32-level sums); only the int8 actions leave it (the library-GEMM version
materialised 3.25 GB of advantages per frame and read them back for the argmax). The update (batch
128 per role, drawn without replacement like random.sample) runs on ms_bdqn_update
(bdqn_update_kernels.hip: the three forwards, the double-DQN target, the MSE backward and the clamp
in eight tile launches) and the HIP Adam, the roles on parallel streams; one frame's updates of all
roles are captured into one HIP graph and replayed.
"""
from __future__ import annotations

import ctypes as ct
import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F_

from . import abi
from ._lib import check, hip_capture, lib, ptr, stream_ptr
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

    def forward(self, x):
        """x [B, obs] float -> q [B, ac_dim, n]."""
        return self.head(F_.linear(x, self.w1, self.b1))

    def hip_params(self) -> abi.MsBdqnParams:
        """ms_bdqn_params of this net (raw device pointers: the parameters change in place, so the struct
        is built once and rebuilt only when the storage moved, e.g. after .to())."""
        key = tuple(getattr(self, k).data_ptr() for k in ("w1", "wa", "ba"))
        if getattr(self, "_hip_key", None) != key:
            self._hip_p = abi.MsBdqnParams(ptr(self.w1), ptr(self.b1), ptr(self.w2), ptr(self.b2), ptr(self.wv),
                                           ptr(self.bv), ptr(self.wa), ptr(self.ba), self.obs, self.ac_dim, self.n)
            self._hip_key = key
        return self._hip_p


class HipActor:
    """get_action of one role on the HIP kernels (bdqn_kernels.hip): the prepared layer 1 (three exact
    bf16 terms of W1; with ``compact`` also b1 + sum_c W1_c F) and the fused act kernel."""

    def __init__(self, q: BranchingQ, seg: int, segs: int, device, compact: bool = False):
        self.q, self.seg, self.segs, self.compact = q, int(seg), int(segs), compact
        self.nbytes = int(lib.ms_bdqn_workspace_bytes(self.seg, self.segs))
        self.ws = torch.empty(((self.nbytes + 3) // 4,), dtype=torch.int32, device=device)
        self.base = torch.empty((128,), dtype=torch.float32, device=device) if compact else None

    def prepare(self, stream=None):
        """After every weight change (the update steps Adam in place)."""
        p = self.q.hip_params()
        check(lib.ms_bdqn_prepare(ct.byref(p), self.seg, self.segs, ptr(self.ws), self.nbytes, ptr(self.base),
                                  stream_ptr(stream)))

    def layer1_compact(self, core_rows, core_owner, n_agents: int, out=None, stream=None):
        """h1 [E * N, 128] of every agent's aggregated acceptor row (ms_bdqn_layer1_compact)."""
        E, C, stride = core_rows.shape
        assert self.compact and C == self.segs and core_rows.dtype == torch.int8 and core_owner.dtype == torch.int8
        assert core_rows.is_contiguous() and core_owner.is_contiguous() and core_owner.shape == (E, C)
        if out is None:
            out = torch.empty((E * n_agents, 128), dtype=torch.float32, device=core_rows.device)
        sb = int(lib.ms_bdqn_layer1_scratch_bytes(E, C))
        if getattr(self, "_scratch", None) is None or self._scratch.numel() * 4 < sb:
            self._scratch = torch.empty(((sb + 3) // 4,), dtype=torch.float32, device=core_rows.device)
        p = self.q.hip_params()
        check(lib.ms_bdqn_layer1_compact(ct.byref(p), ptr(self.ws), ptr(self.base), ptr(core_rows), ptr(core_owner), E,
                                         n_agents, C, self.seg, stride, ptr(self._scratch), self._scratch.numel() * 4,
                                         ptr(out), stream_ptr(stream)))
        return out

    def act_compact(self, core_rows, core_owner, n_agents: int, explore=None, rand_action=None, out=None, stream=None):
        """ms_bdqn_act_compact: the acceptor role's actions [E * N, ac_dim] int8 straight from the compact
        observations (layer 1 summed in the act kernel, no h1 rows); equal to act(h1=layer1_compact(...))."""
        E, C, stride = core_rows.shape
        assert self.compact and C == self.segs and core_rows.dtype == torch.int8 and core_owner.dtype == torch.int8
        assert core_rows.is_contiguous() and core_owner.is_contiguous() and core_owner.shape == (E, C)
        rows = E * n_agents
        if explore is not None:
            assert explore.dtype == torch.uint8 and explore.numel() == rows
            assert rand_action.dtype == torch.int8 and rand_action.shape == (rows, self.q.ac_dim)
            assert rand_action.is_contiguous()
        if out is None:
            out = torch.empty((rows, self.q.ac_dim), dtype=torch.int8, device=core_rows.device)
        sb = int(lib.ms_bdqn_layer1_scratch_bytes(E, C))
        if getattr(self, "_scratch", None) is None or self._scratch.numel() * 4 < sb:
            self._scratch = torch.empty(((sb + 3) // 4,), dtype=torch.float32, device=core_rows.device)
        p = self.q.hip_params()
        check(lib.ms_bdqn_act_compact(ct.byref(p), ptr(self.ws), ptr(self.base), ptr(core_rows), ptr(core_owner), E,
                                      n_agents, C, self.seg, stride, ptr(self._scratch), self._scratch.numel() * 4,
                                      ptr(explore), ptr(rand_action), ptr(out), stream_ptr(stream)))
        return out

    def act(self, h1=None, x=None, explore=None, rand_action=None, out=None, stream=None):
        """ms_bdqn_act: int8 [rows, ac_dim] actions from h1 [rows, 128] f32 or int8 rows x [rows, stride]."""
        src = h1 if h1 is not None else x
        rows = src.shape[0]
        assert src.is_contiguous()
        if h1 is not None:
            assert h1.dtype == torch.float32 and h1.shape[1] == 128
        else:
            assert x.dtype == torch.int8 and x.shape[1] >= self.q.obs and self.segs == 1
        if explore is not None:
            assert explore.dtype == torch.uint8 and explore.numel() == rows
            assert rand_action.dtype == torch.int8 and rand_action.shape == (rows, self.q.ac_dim)
            assert rand_action.is_contiguous()
        if out is None:
            out = torch.empty((rows, self.q.ac_dim), dtype=torch.int8, device=src.device)
        p = self.q.hip_params()
        check(lib.ms_bdqn_act(ct.byref(p), ptr(h1), ptr(x), 0 if x is None else x.shape[1],
                              ptr(self.ws) if x is not None else None, rows, ptr(explore), ptr(rand_action), ptr(out),
                              stream_ptr(stream)))
        return out


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
    graph_updates: bool = True   # BranchingRole updates replayed from a captured HIP graph
    hip_updates: bool = True     # update_policy on ms_bdqn_update (else torch autograd, the reference form)

    def epsilon_by_frame(self, i):
        return self.epsilon_final + (self.epsilon_start - self.epsilon_final) * math.exp(-1.0 * i / self.epsilon_decay)


class BranchingRole:
    """BranchingDQN (BranchingDQNModules.py:104-164) of one role: online / target nets, Adam, counter.

    With ``graph`` the update's ~80 small launches (three forwards, the loss, the backward, the
    clamp and the HIP Adam) are captured once into a HIP graph and replayed on static input
    buffers: the batch is 128 rows, so the eager update is launch-bound, not compute-bound. The
    first update runs eagerly (on a side stream, torch's capture recipe) and is this step's real
    update; the target sync stays on the host every target_net_update_freq updates (an in-place
    copy into the tensors the graph reads)."""

    def __init__(self, obs: int, ac_dim: int, n: int, cfg: BDQNConfig, device, graph: bool = False):
        self.q = BranchingQ(obs, ac_dim, n).to(device)
        self.target = BranchingQ(obs, ac_dim, n).to(device)  # its own init draw, then overwritten (:110-112)
        self.target.load_state_dict(self.q.state_dict())
        self.target.requires_grad_(False)
        self.cfg = cfg
        self.opt = HipAdam([dict(params=list(self.q.parameters()), lr=cfg.lr)])
        self.update_counter = 0
        self.graph = graph
        self._g = None

    def _body(self, states, actions, rewards, next_states, masks):
        current = self.q(states).gather(2, actions.unsqueeze(2)).squeeze(-1)
        with torch.no_grad():
            argmax = torch.argmax(self.q(next_states), dim=2)
            max_next = self.target(next_states).gather(2, argmax.unsqueeze(2)).squeeze(-1).mean(1, keepdim=True)
        expected = rewards.view(-1, 1) + max_next * self.cfg.gamma * masks.view(-1, 1)
        loss = ((expected - current) ** 2).mean()  # F.mse_loss(expected, current) broadcast over branches
        for p in self.q.parameters():  # optimizer.zero_grad(), in place (the graph keeps the .grad tensors)
            if p.grad is not None:
                p.grad.zero_()
        loss.backward()
        if self.cfg.grad_clip > 0:  # grad_clip <= 0: no clamp (the ms_bdqn_update convention)
            for p in self.q.parameters():
                p.grad.data.clamp_(-self.cfg.grad_clip, self.cfg.grad_clip)
        self.opt.step()
        return loss.detach()

    def hip_update(self, states_i8, next_i8, actions_i8, rewards, masks, stream=None):
        """update_policy (BranchingDQNModules.py:125-164) on the HIP kernels (ms_bdqn_update: the three
        forwards, the double-DQN target, the MSE backward and the clamp in eight tile launches) and the HIP
        Adam: states / next states [B, ld] int8 observation rows, actions [B, >= ac_dim] int8, rewards /
        masks [B] f32. Capturable (no host sync). Returns the loss tensor [1] (overwritten by the
        next update)."""
        B = states_i8.shape[0]
        for x in (states_i8, next_i8, actions_i8):
            assert x.dtype == torch.int8 and x.is_contiguous() and x.shape[0] == B
        assert rewards.dtype == torch.float32 and masks.dtype == torch.float32
        assert rewards.is_contiguous() and masks.is_contiguous() and rewards.numel() == masks.numel() == B
        q = self.q
        if getattr(self, "_upd_ws", None) is None:
            nb = int(lib.ms_bdqn_update_workspace_bytes(ct.byref(q.hip_params()), 128))
            self._upd_ws = torch.empty(((nb + 3) // 4,), dtype=torch.float32, device=states_i8.device)
            self._upd_loss = torch.zeros((1,), dtype=torch.float32, device=states_i8.device)
            for prm in q.parameters():
                if prm.grad is None:
                    prm.grad = torch.zeros_like(prm)
        qp, tp = q.hip_params(), self.target.hip_params()
        bt = abi.MsBdqnBatch(ptr(states_i8), ptr(next_i8), states_i8.shape[1], ptr(actions_i8), actions_i8.shape[1],
                             ptr(rewards), ptr(masks), B)
        gr = abi.MsBdqnGrads(*[ptr(getattr(q, k).grad) for k in KEYS], ptr(self._upd_loss))
        check(lib.ms_bdqn_update(ct.byref(qp), ct.byref(tp), ct.byref(bt), ct.c_float(self.cfg.gamma),
                                 ct.c_float(self.cfg.grad_clip), ptr(self._upd_ws), self._upd_ws.numel() * 4,
                                 ct.byref(gr), stream_ptr(stream)))
        self.opt.step(stream)
        return self._upd_loss

    def count_update(self):
        """update_counter and the target sync of update_policy (:161-164), on the host."""
        self.update_counter += 1
        if self.update_counter % self.cfg.target_net_update_freq == 0:
            self.update_counter = 0
            with torch.no_grad():
                for k in KEYS:
                    getattr(self.target, k).copy_(getattr(self.q, k))

    def update(self, states, actions, rewards, next_states, masks):
        """update_policy (BranchingDQNModules.py:125-164) in torch autograd (the numerical reference of
        hip_update) on a drawn batch: states / next_states [B, obs] float, actions [B, ac_dim] long,
        rewards / masks [B]. Returns the loss."""
        if not self.graph:
            loss = self._body(states, actions, rewards, next_states, masks)
        elif self._g is None:
            self._in = [x.detach().clone() for x in (states, actions, rewards, next_states, masks)]
            side = torch.cuda.Stream(device=states.device)
            side.wait_stream(torch.cuda.current_stream(states.device))
            with torch.cuda.stream(side):
                loss = self._body(*self._in).clone()  # this step's update (and the warm-up of the capture)
            torch.cuda.current_stream(states.device).wait_stream(side)
            torch.cuda.synchronize(states.device)
            g = torch.cuda.CUDAGraph()
            with hip_capture(g):
                self._loss = self._body(*self._in)
            self._g = g
        else:
            for dst, src in zip(self._in, (states, actions, rewards, next_states, masks)):
                dst.copy_(src)
            self._g.replay()
            loss = self._loss.clone()
        self.update_counter += 1
        if self.update_counter % self.cfg.target_net_update_freq == 0:
            self.update_counter = 0
            self.target.load_state_dict(self.q.state_dict())
        return loss


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
        self.seed = int(seed)
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
        gr = self.b.graph_updates
        self.roles = dict(acc=BranchingRole(C * s.acc_obs_dim, C, O + 1, self.b, dev, graph=gr),
                          off=BranchingRole(self.d_off, L, C + 1, self.b, dev, graph=gr))
        if self.free:
            self.roles["price"] = BranchingRole(self.d_off, L, s.price_actions, self.b, dev, graph=gr)
        # acting on the HIP kernels: the acceptor's layer 1 from the compact rows, the offer / price
        # roles' on the aggregated offer rows inside the act kernel
        self.actors = {k: (HipActor(r.q, self.d_acc, C, dev, compact=True) if k == "acc"
                           else HipActor(r.q, self.d_off, 1, dev)) for k, r in self.roles.items()}
        # compact replay ring: states of frames 0..F (slot F + 1 holds the next state of the newest frame)
        Fm = self.b.memory_frames
        self.n_slots = Fm + 1
        E = self.E
        self.core_rows = torch.zeros((self.n_slots, E, C, self.stride), dtype=torch.int8, device=dev)
        self.core_owner = torch.zeros((self.n_slots, E, C), dtype=torch.int8, device=dev)
        self.slot_pairs = torch.zeros((self.n_slots, E, N, L, 2), dtype=torch.int8, device=dev)
        self.act = {k: torch.zeros((self.n_slots, E, N, r.q.ac_dim), dtype=torch.int8, device=dev)
                    for k, r in self.roles.items()}
        # the aggregated acceptor / offer rewards are int32 (Reward.py:92-143) and the env kernel writes
        # them straight into the ring slot; the price role's float sums are copied in
        self.rew = {k: torch.zeros((self.n_slots, E, N), dtype=torch.float32 if k == "price" else torch.int32,
                                   device=dev) for k in self.roles}
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
        self.timings = None

    def _observe_into(self, slot, reset=False):
        obs = dict(core_rows=self.core_rows[slot], core_owner=self.core_owner[slot], offer=self.off_rows)
        if reset:
            self.env.reset(obs)
        return obs

    def _store_slot_pairs(self, slot):
        self.slot_pairs[slot].copy_(self.off_rows[..., 2 * self.C:2 * self.C + 2])

    def _offer_rows_i8(self, slot):
        """The aggregated offer rows [E * N, ld_off] int8 of every (replica, agent) of ring slot `slot`
        (ms_regen_agent_rows)."""
        E, N = self.E, self.N
        if getattr(self, "_frame_base", None) is None:
            self._frame_base = torch.arange(E, device=self.device, dtype=torch.int64).repeat_interleave(N)
        frame = self._frame_base + slot * E
        _, off = self.env.regen_agent_rows(self.core_rows.view(-1, self.C, self.stride),
                                           self.core_owner.view(-1, self.C), self.slot_pairs.view(-1, N, self.L, 2),
                                           frame, self._agent_idx,
                                           offer=torch.empty((E * N, self.ld_off), dtype=torch.int8,
                                                             device=self.device))
        return off

    @torch.no_grad()
    def _actions(self, slot, eps):
        """get_action (BranchingDQNModules.py:117-123) of every agent, epsilon-greedy per agent (:181-186):
        one fused HIP act kernel per role (ms_bdqn_act; the acceptor role ms_bdqn_act_compact)."""
        E, N = self.E, self.N
        for a in self.actors.values():
            a.prepare()  # the weights changed in the last update
        x_off = self._offer_rows_i8(slot)
        explore = torch.empty((E * N,), dtype=torch.uint8, device=self.device).bernoulli_(eps, generator=self.gen)
        out = {}
        for k, actor in self.actors.items():
            q = actor.q
            rnd = torch.randint(0, q.n, (E * N, q.ac_dim), generator=self.gen, device=self.device, dtype=torch.int8)
            dst = self.act[k][slot].view(E * N, q.ac_dim)  # written in place: the ring slot of this frame
            if k == "acc":  # layer 1 from the compact frame, summed inside the act kernel
                a = actor.act_compact(self.core_rows[slot], self.core_owner[slot], N, explore=explore, rand_action=rnd,
                                      out=dst)
            else:
                a = actor.act(x=x_off, explore=explore, rand_action=rnd, out=dst)
            out[k] = a.view(E, N, -1)
        return out

    @property
    def timings(self):
        """Device time (s) of the frames' acting, env step + storing, and learning, accumulated from
        HIP events (read lazily)."""
        self._fold_events(block=True)
        return self._timings

    def _fold_events(self, block: bool, keep: int = 0):
        """Add the pending frames' event spans to the timings, oldest first: all of them (block), or
        those already complete plus any beyond the newest ``keep`` (each step folds with keep = 32,
        so a long run holds a bounded number of HIP events)."""
        while self._pending_events:
            ev = self._pending_events[0]
            if not block and len(self._pending_events) <= keep and not ev[-1].query():
                break
            ev[-1].synchronize()
            self._timings["act"] += ev[0].elapsed_time(ev[1]) / 1e3
            self._timings["env"] += ev[1].elapsed_time(ev[2]) / 1e3
            self._timings["learn"] += ev[2].elapsed_time(ev[3]) / 1e3
            self._event_pool.append(self._pending_events.pop(0))  # reused: no new HIP events per frame

    @timings.setter
    def timings(self, value):
        self._pending_events = []
        self._event_pool = []
        self._timings = dict(act=0.0, env=0.0, learn=0.0)

    def step(self):
        """One frame: act, env.step, store the transition, learn (BranchingDQNModules.py:179-208)."""
        E, N, C, L = self.E, self.N, self.C, self.L
        b = self.b
        cur = self.head
        nxt = (cur + 1) % self.n_slots
        eps = b.epsilon_by_frame(self.frame)
        ev = self._event_pool.pop() if self._event_pool else [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        if self.frame + 1 > b.learning_starts and b.hip_updates and not getattr(self, "_staged", False):
            # this frame's minibatch (after this frame's store: stored + 1 frames, head nxt); from the
            # second learning frame on it was drawn during the previous step
            self._draw_sample(min(self.stored + 1, b.memory_frames), nxt)
            self._queue_sample()
            self._staged = True
        ev[0].record()
        acts = self._actions(cur, eps)
        ev[1].record()
        if self.frame + 2 > b.learning_starts and b.hip_updates:
            # the next frame's minibatch drawn on the host now, while the device runs this frame's
            # acting; its copy is queued after this frame's learn (which still reads the index buffer)
            self._draw_sample(min(min(self.stored + 1, b.memory_frames) + 1, b.memory_frames),
                              (nxt + 1) % self.n_slots)
        obs = self._observe_into(nxt)
        price = acts["price"].contiguous() if self.free else None
        rew = dict(self.rbuf)
        rew["aggregated_acceptor"] = self.rew["acc"][cur]  # written in place by the step kernel
        rew["aggregated_offer"] = self.rew["off"][cur]
        self.env.step(acts["acc"].contiguous(), acts["off"].contiguous(), price, obs=obs, rewards=rew)
        self._store_slot_pairs(nxt)
        done = self.env.round % self.cfg.episode_length == 0
        if self.free:
            self.rew["price"][cur].copy_(rew["price"].sum(2))
        self.mask[cur] = 0.0 if done else 1.0
        self.head = nxt
        self.stored = min(self.stored + 1, self.b.memory_frames)
        self.frame += 1
        ev[2].record()
        if self.frame > b.learning_starts:
            self._learn()
        ev[3].record()
        self._staged = False
        if getattr(self, "_drawn", None) is not None:
            self._queue_sample()
            self._staged = True
        self._pending_events.append(ev)
        self._fold_events(block=False, keep=32)
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

    def _sample_host(self, stored=None, head=None):
        """batch_size transitions drawn without replacement from the stored frames' E x N transitions,
        as random.sample(memory, batch_size) (BranchingDQNModules.py:53-55) on a host random.Random:
        [4][B] int64 (ring record, next record, agent, ring slot), 0 = the newest stored frame."""
        import random

        import numpy as np

        E, N, B = self.E, self.N, self.b.batch_size
        if getattr(self, "_py_rng", None) is None:
            self._py_rng = random.Random(self.seed + 29)
        stored = self.stored if stored is None else stored
        head = self.head if head is None else head
        js = np.array(self._py_rng.sample(range(stored * E * N), B), dtype=np.int64)
        age, rest = np.divmod(js, E * N)
        e, a = np.divmod(rest, N)
        slot = (head - 1 - age) % self.n_slots
        return np.stack([slot * E + e, ((slot + 1) % self.n_slots) * E + e, a, slot])

    def _learn(self):
        if self.b.hip_updates:
            return self._learn_hip()
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
            r = self.rew[k][slot, e, a.long()].float()
            losses[k] = role.update(s, acts, r, s1, masks)
        self.last_losses = losses

    def _learn_body(self):
        """One frame's updates from the drawn indices in self._sel (device): the minibatch's rows
        regenerated from the compact frames (ms_regen_agent_rows), the actions / rewards / masks
        gathered, then every role's ms_bdqn_update + HIP Adam. No host sync: captured once, replayed."""
        C, N, L = self.C, self.N, self.L
        rec, nrec, a, slot = self._sel[0], self._sel[1], self._sel[2], self._sel[3]
        a32 = a.to(torch.int32)
        cr = self.core_rows.view(-1, C, self.stride)
        co = self.core_owner.view(-1, C)
        sp = self.slot_pairs.view(-1, N, L, 2)
        acc_s, off_s = self.env.regen_agent_rows(cr, co, sp, rec, a32)
        acc_n, off_n = self.env.regen_agent_rows(cr, co, sp, nrec, a32)
        xs = dict(acc=(acc_s, acc_n), off=(off_s, off_n))
        xs["price"] = xs["off"]
        masks = self.mask[slot]
        flat = rec * N + a
        losses = {}
        # the roles' updates are independent chains of small launches (a 128-row batch): one stream
        # each, forked from and joined back into the current stream (captured as parallel branches)
        main = torch.cuda.current_stream(self.device)
        if getattr(self, "_role_streams", None) is None:
            self._role_streams = {k: torch.cuda.Stream(device=self.device) for k in self.roles}
        for k, role in self.roles.items():
            st = self._role_streams[k]
            st.wait_stream(main)
            with torch.cuda.stream(st):
                s, s1 = xs[k]
                acts = self.act[k].view(-1, role.q.ac_dim)[flat]
                r = self.rew[k].view(-1)[flat].float()
                losses[k] = role.hip_update(s, s1, acts, r, masks)
        for st in self._role_streams.values():
            main.wait_stream(st)
        return losses

    def _draw_sample(self, stored, head):
        """Draw a frame's minibatch on the host into the next pinned staging buffer (two alternate: the
        buffer's previous copy, two frames ago, is long done)."""
        B = self.b.batch_size
        if getattr(self, "_sel", None) is None:
            self._sel_hosts = [torch.empty((4, B), dtype=torch.int64, pin_memory=True) for _ in range(2)]
            self._sel_events = [torch.cuda.Event() for _ in range(2)]
            self._sel_flip = 0
            self._sel = torch.empty((4, B), dtype=torch.int64, device=self.device)
            self._learn_graph = None
        i = self._sel_flip
        self._sel_flip ^= 1
        self._sel_events[i].synchronize()
        self._sel_host = self._sel_hosts[i]
        self._sel_host.copy_(torch.from_numpy(self._sample_host(stored, head)))
        self._drawn = i

    def _queue_sample(self):
        """Queue the drawn minibatch's copy to the device index buffer the learn graph reads (stream order
        puts it after the previous learn)."""
        i = self._drawn
        self._sel.copy_(self._sel_hosts[i], non_blocking=True)
        self._sel_events[i].record()
        self._drawn = None

    def _learn_hip(self):
        if not self.b.graph_updates:
            self.last_losses = self._learn_body()
        elif self._learn_graph is None:
            self.last_losses = self._learn_body()  # this frame's updates (and the capture's warm-up)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with hip_capture(g):
                self._graph_losses = self._learn_body()
            self._learn_graph = g
        else:
            self._learn_graph.replay()
            self.last_losses = self._graph_losses
        for role in self.roles.values():
            role.count_update()

    def flags(self) -> int:
        return self.env.flags()
