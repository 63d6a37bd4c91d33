"""DQN units of the reference (DQNmodules.py) batched over groups and env replicas, and the batched
DQN training loop of trainDQN.py (DQNDividedFixedPricesEnv, SchedulingEnvironment.py:351-436).

The reference gives every unit of every agent its own DQNEntity (Linear(D,16)-Tanh-Linear(16,A),
DQNmodules.py:34-94) with a target copy, an Adam optimizer and a ReplayMemory
(DividedFixPriceDQNAgent Agent.py:303-356). Each round it pushes (s, a, s', r) into every unit's
memory and runs optimize_model on it (DQNmodules.py:97-154): BATCH_SIZE transitions drawn with
replacement, SmoothL1 between Q(s)[a] and r + GAMMA * max Q_target(s'), every gradient element
clamped to [-1, 1], Adam with torch's defaults. Here the G nets of one unit type serve all E
replicas: acting is one ``ms_dqn_act`` launch, a round's optimisation is one ``ms_dqn_grad`` launch
(each replica samples its own minibatch from its own memory; the loss is the replicas' mean, so
E = 1 is the reference) plus one ``ms_adam_step``.
"""
from __future__ import annotations

import ctypes as ct
import math
from dataclasses import dataclass

import torch
import torch.nn as nn

from . import abi
from ._lib import check, lib, ptr, stream_ptr
from .ppo import HipAdam

HIDDEN = 16  # DQNEntity (DQNmodules.py:41-46)
KEYS = ("w1", "b1", "w2", "b2")


def reference_qnet_params(in_dim: int, n_actions: int):
    """One DQNEntity initialised like the reference: Linear(D, 16) then Linear(16, A) on the current
    torch CPU generator (DQNmodules.py:41-46). The target net is a deepcopy (Agent.py:310): no draw."""
    l1, l2 = nn.Linear(in_dim, HIDDEN), nn.Linear(HIDDEN, n_actions)
    return dict(w1=l1.weight, b1=l1.bias, w2=l2.weight, b2=l2.bias)


def reference_dqn_nets(N: int, C: int, L: int, dims: dict):
    """DividedFixPriceDQNAgent construction order (Agent.py:306-309): agent by agent, C acceptor nets
    then L offer nets. dims: acc/off -> (D, A). Returns name -> [param dict per unit]."""
    nets = dict(acc=[], off=[])
    for _ in range(N):
        for _ in range(C):
            nets["acc"].append(reference_qnet_params(*dims["acc"]))
        for _ in range(L):
            nets["off"].append(reference_qnet_params(*dims["off"]))
    return nets


class GroupedQNet(nn.Module):
    """G DQNEntity nets of one shape, parameters stacked along dim 0."""

    def __init__(self, nets: list, in_dim: int, n_actions: int):
        super().__init__()
        self.G, self.D, self.A = len(nets), in_dim, n_actions
        for k in KEYS:
            self.register_parameter(k, nn.Parameter(torch.stack([n[k].detach() for n in nets]).contiguous()))

    def forward(self, x):
        """x [G, R, D] float -> Q [G, R, A] (torch, for checks)."""
        h = torch.tanh(torch.baddbmm(self.b1.unsqueeze(1), x, self.w1.transpose(1, 2)))
        return torch.baddbmm(self.b2.unsqueeze(1), h, self.w2.transpose(1, 2))

    def params(self) -> abi.MsQnetParams:
        for k in KEYS:
            t = getattr(self, k)
            assert t.is_cuda and t.is_contiguous() and t.dtype == torch.float32
        return abi.MsQnetParams(ptr(self.w1), ptr(self.b1), ptr(self.w2), ptr(self.b2), self.D, HIDDEN, self.A, self.G)

    @torch.no_grad()
    def act(self, obs_i8, units_per_group: int, eps: float, seed: int = 0, offset: int = 0, uniforms=None,
            action=None, greedy=None, offset_dev=None, stream=None):
        """selectAction (DQNmodules.py:56-70) for obs [E, U, stride] int8: greedy = first argmax of Q;
        action = greedy where the row's uniform u1 > eps, else floor(u2 * A). uniforms: [2, E, U]
        float64 or None (Philox). Returns (action, greedy) int8 [E, U]."""
        E, U, stride = obs_i8.shape
        assert obs_i8.dtype == torch.int8 and obs_i8.is_contiguous() and U == units_per_group * self.G
        dev = obs_i8.device
        action = torch.empty((E, U), dtype=torch.int8, device=dev) if action is None else action
        greedy = torch.empty((E, U), dtype=torch.int8, device=dev) if greedy is None else greedy
        if uniforms is not None:
            assert uniforms.dtype == torch.float64 and uniforms.is_contiguous() and uniforms.numel() == 2 * E * U
        p = self.params()
        check(lib.ms_dqn_act(ct.byref(p), ptr(obs_i8), stride, E, U, units_per_group, ct.c_double(eps), ptr(uniforms),
                             ct.c_uint64(seed), ct.c_uint64(offset), ptr(offset_dev), ptr(action), ptr(greedy),
                             stream_ptr(stream)))
        return action, greedy


class ReplayMemories:
    """ReplayMemory (DQNmodules.py:13-31) of every (replica, unit) of one unit type on the device:
    transitions (state row, action, next-state row, reward) in [E][U][capacity]. All memories of a
    run receive one push per round, so nextFreeIndex is one host integer; the replacement index of a
    full memory (random.randint(0, capacity - 1)) is drawn per memory."""

    def __init__(self, E: int, U: int, capacity: int, stride: int, device):
        assert capacity >= 2
        self.E, self.U, self.cap, self.stride = E, U, capacity, stride
        self.states = torch.zeros((E, U, capacity, stride), dtype=torch.int8, device=device)
        self.next_states = torch.zeros_like(self.states)
        self.actions = torch.zeros((E, U, capacity), dtype=torch.int8, device=device)
        self.rewards = torch.zeros((E, U, capacity), dtype=torch.float32, device=device)
        self.next_free = 0

    def _put(self, idx, s, a, r, s1):
        """Transition of every memory at index idx (int, or [E, U] long tensor)."""
        if isinstance(idx, int):
            self.states[:, :, idx].copy_(s)
            self.next_states[:, :, idx].copy_(s1)
            self.actions[:, :, idx].copy_(a)
            self.rewards[:, :, idx].copy_(r)
            return
        i3 = idx.unsqueeze(-1)
        i4 = i3.unsqueeze(-1).expand(-1, -1, 1, self.stride)
        self.states.scatter_(2, i4, s.unsqueeze(2))
        self.next_states.scatter_(2, i4, s1.unsqueeze(2))
        self.actions.scatter_(2, i3, a.unsqueeze(2))
        self.rewards.scatter_(2, i3, r.unsqueeze(2).to(torch.float32))

    def push(self, s, a, r, s1, replace_index=None):
        """ReplayMemory.push (DQNmodules.py:19-25): while nextFreeIndex + 1 < capacity the transition goes
        to nextFreeIndex; once nextFreeIndex + 1 == capacity (after that first branch too) it also
        overwrites memory[random.randint(0, capacity - 1)]. replace_index: callable -> [E, U] long
        (drawn only when needed). s, s1 [E, U, stride] int8; a [E, U] int8; r [E, U]."""
        if self.next_free + 1 < self.cap:
            self._put(self.next_free, s, a, r, s1)
            self.next_free += 1
        if self.next_free + 1 == self.cap:
            self._put(replace_index(), s, a, r, s1)


@dataclass
class DQNHyper:
    """RL parameters of trainDQN.py:72-99."""
    batch_size: int = 10
    offer_gamma: float = 0.5
    acceptor_gamma: float = 0.84
    run_start: float = 0.9
    run_end: float = 0.05
    run_decay: float = 500
    replay_memory_size: int = 5000
    target_update: int = 2      # episodes between target syncs (trainDQN.py:266-268)
    lr: float = 1e-3            # optim.Adam(net.parameters()) defaults (Agent.py:312-319)
    random_policy: bool = False
    grad_clip: float = 1.0      # p.grad.data.clamp_(-1, 1) (DQNmodules.py:151-152)


def epsilon(hp: DQNHyper, world_round: int) -> float:
    """eps_treshold of DQNEntity.selectAction (DQNmodules.py:61-63)."""
    return hp.run_end + (hp.run_start - hp.run_end) * math.exp(-1.0 * world_round / hp.run_decay)


class DQNGroup:
    """Policy / target nets, Adam and the replay memories of one unit type."""

    def __init__(self, nets: list, in_dim: int, n_actions: int, gamma: float, hp: DQNHyper, device):
        self.policy = GroupedQNet(nets, in_dim, n_actions).to(device)
        self.target = GroupedQNet(nets, in_dim, n_actions).to(device)
        self.target.requires_grad_(False)
        self.gamma, self.hp = gamma, hp
        self.opt = HipAdam([dict(params=list(self.policy.parameters()), lr=hp.lr)])
        for p in self.policy.parameters():
            p.grad = torch.zeros_like(p)
        self.loss = torch.zeros(self.policy.G, dtype=torch.float32, device=device)
        self._ws = None

    @torch.no_grad()
    def sync_target(self):
        """target.load_state_dict(policy.state_dict()) (Agent.py:329-334)."""
        for k in KEYS:
            getattr(self.target, k).copy_(getattr(self.policy, k))

    def grad(self, mem: ReplayMemories, samples, units_per_group: int = 1, stream=None, clip: float | None = None):
        """The minibatch gradient of every group (ms_dqn_grad) into policy's .grad, clamped to
        +-clip (default hp.grad_clip; inf = unclamped, for a multi-rank step that clamps the mean)."""
        E, U, B = samples.shape
        assert samples.dtype == torch.int32 and samples.is_contiguous() and U == mem.U and E == mem.E
        pp, tp = self.policy.params(), self.target.params()
        rows = units_per_group * E * B
        need = lib.ms_dqn_workspace_bytes(ct.byref(pp), rows)
        if self._ws is None or self._ws.numel() * 4 < need:
            self._ws = torch.empty(((need + 3) // 4,), dtype=torch.float32, device=samples.device)
        b = abi.MsDqnBatch(ptr(mem.states), ptr(mem.next_states), ptr(mem.actions), ptr(mem.rewards), ptr(samples),
                           mem.stride, U, units_per_group, mem.cap, B, E, ct.c_float(self.gamma))
        pol = self.policy
        g = abi.MsQnetGrads(ptr(pol.w1.grad), ptr(pol.b1.grad), ptr(pol.w2.grad), ptr(pol.b2.grad), ptr(self.loss))
        check(lib.ms_dqn_grad(ct.byref(pp), ct.byref(tp), ct.byref(b), ct.c_float(self.hp.grad_clip if clip is None else clip), ptr(self._ws),
                              self._ws.numel() * 4, ct.byref(g), stream_ptr(stream)))
        return self.loss

    def optimize(self, mem: ReplayMemories, samples, units_per_group: int = 1, stream=None):
        """optimize_model (DQNmodules.py:97-154) of every group: gradient, then Adam."""
        loss = self.grad(mem, samples, units_per_group, stream).clone()
        self.opt.step(stream)
        return loss


class DQNTrainer:
    """trainDQN.py:126-268 over E replicas of DQNDividedFixedPricesEnv (SchedulingEnvironment.py:428-436).

    One ``episode()`` = episodeLength rounds of: selectAction of every unit (offer nets, acceptor nets;
    epsilon from world.round) -> env.step with the in-kernel hard-coded auctioneer -> unless the
    round ends the episode, push (s, a, s', r) into every unit's memory and optimise every unit
    (updateAcceptorMemoriesAndOptimize, updateOfferMemoriesAndOptimize :366-425). After episode i
    with i % TARGET_UPDATE == 0 the target nets are synced. Random streams: epsilon / exploration
    uniforms from Philox (per rank, round, unit), memory replacement indices and minibatch samples
    from a torch device generator; the env stream stays the reference's per replica."""

    def __init__(self, cfg: abi.MsConfig, n_envs: int, hyper: DQNHyper | None = None, seed: int = 0, device=None,
                 episode_length: int | None = None, rank: int = 0, world_size: int = 1, process_group=None):
        from .env import BatchedEnv
        from .trainer import allreduce_mean_grads, env_seed
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        torch.cuda.set_device(self.device)
        if cfg.free_prices:
            raise ValueError("the DQN env is fixed-price only (DQNDividedFixedPricesEnv, SchedulingEnvironment.py:428)")
        if episode_length is not None:
            cfg = abi.MsConfig.from_buffer_copy(cfg)
            cfg.episode_length = int(episode_length)
        self.cfg, self.E, self.hp = cfg, int(n_envs), hyper or DQNHyper()
        self.rank, self.world_size, self.pg = rank, world_size, process_group
        self._allreduce = (lambda ps: allreduce_mean_grads(ps, world_size, process_group)) if world_size > 1 else None
        self.env = BatchedEnv(cfg, self.E, seed=env_seed(seed, rank, self.E), device=self.device)
        s = self.env.shape
        N, C, L = s.n_agents, s.n_cores, s.collection_length
        self.N, self.C, self.L = N, C, L
        self.ep_len = int(cfg.episode_length)
        torch.manual_seed(seed)
        nets = reference_dqn_nets(N, C, L, dict(acc=(s.acc_obs_dim, s.acc_actions), off=(s.off_obs_dim, s.off_actions)))
        dev, hp = self.device, self.hp
        self.acc = DQNGroup(nets["acc"], s.acc_obs_dim, s.acc_actions, hp.acceptor_gamma, hp, dev)
        self.off = DQNGroup(nets["off"], s.off_obs_dim, s.off_actions, hp.offer_gamma, hp, dev)
        if world_size > 1:
            import torch.distributed as dist
            for grp in (self.acc, self.off):
                for p in grp.policy.parameters():
                    dist.broadcast(p.data, src=0, group=process_group)
                grp.sync_target()
        cap = hp.replay_memory_size
        self.mem_acc = ReplayMemories(self.E, N * C, cap, s.acc_obs_stride, dev)
        self.mem_off = ReplayMemories(self.E, N * L, cap, s.off_obs_stride, dev)
        # current / next observation buffers (ping-pong)
        self.obs = [dict(acceptor=torch.zeros((self.E, N * C, s.acc_obs_stride), dtype=torch.int8, device=dev),
                         offer=torch.zeros((self.E, N * L, s.off_obs_stride), dtype=torch.int8, device=dev))
                    for _ in range(2)]
        self.cur = 0
        self.env.reset({k: v.view(self.E, N, -1, v.shape[-1]) for k, v in self.obs[0].items()})
        self.rew = dict(offer=torch.zeros((self.E, N, L), dtype=torch.float32, device=dev),
                        acceptor=torch.zeros((self.E, N, C), dtype=torch.int32, device=dev),
                        agent=torch.zeros((self.E, N), dtype=torch.int32, device=dev),
                        auctioneer=torch.zeros((self.E, C), dtype=torch.int32, device=dev))
        self.act_acc = torch.zeros((self.E, N * C), dtype=torch.int8, device=dev)
        self.act_off = torch.zeros((self.E, N * L), dtype=torch.int8, device=dev)
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed * 7919 + rank)
        self.seed = seed
        self.episodes = 0
        self.last_losses = {}

    @property
    def round(self) -> int:
        return self.env.round

    def _replace_index(self, mem):
        return lambda: torch.randint(0, mem.cap, (mem.E, mem.U), generator=self.gen, device=self.device)

    def _samples(self, mem):
        return torch.randint(0, mem.next_free, (mem.E, mem.U, self.hp.batch_size), generator=self.gen,
                             device=self.device, dtype=torch.int32)

    def _optimize(self):
        """updateAcceptorMemoriesAndOptimize then updateOfferMemoriesAndOptimize (SchedulingEnvironment.py:366-425)
        for all units at once; with several ranks one all-reduce carries both unit types' gradients."""
        grads = {}
        # several ranks: clamp the rank-averaged gradient (DQNmodules.py:151-152 clamps the gradient
        # of the whole minibatch), not each rank's share, so results do not depend on the rank count
        multi = self._allreduce is not None
        for name, grp, mem in (("acc", self.acc, self.mem_acc), ("off", self.off, self.mem_off)):
            grads[name] = grp.grad(mem, self._samples(mem), clip=float("inf") if multi else None).clone()
        if multi:
            params = list(self.acc.policy.parameters()) + list(self.off.policy.parameters())
            self._allreduce(params)
            for p in params:
                p.grad.clamp_(-self.hp.grad_clip, self.hp.grad_clip)
        for grp in (self.acc, self.off):
            grp.opt.step()
        self.last_losses = grads

    def step_round(self):
        """One round of the trainDQN.py loop body; returns done."""
        N, C, L, E = self.N, self.C, self.L, self.E
        s, s1 = self.obs[self.cur], self.obs[1 - self.cur]
        r = self.round
        eps = 2.0 if self.hp.random_policy else epsilon(self.hp, r)  # randomPolicy: always explore
        key = self.seed * 7919 + self.rank
        # getActions: offer nets then acceptor nets per agent (Agent.py:345-356); Philox per unit type
        self.off.policy.act(s["offer"], 1, eps, seed=key, offset=4 * r + 1, action=self.act_off)
        self.acc.policy.act(s["acceptor"], 1, eps, seed=key, offset=4 * r + 2, action=self.act_acc)
        obs_out = {k: v.view(E, N, -1, v.shape[-1]) for k, v in s1.items()}
        self.env.step(self.act_acc.view(E, N, C), self.act_off.view(E, N, L), obs=obs_out, rewards=self.rew)
        done = self.round % self.ep_len == 0
        if not done and not self.hp.random_policy:
            self.mem_acc.push(s["acceptor"], self.act_acc, self.rew["acceptor"].view(E, N * C), s1["acceptor"],
                              self._replace_index(self.mem_acc))
            self.mem_off.push(s["offer"], self.act_off, self.rew["offer"].view(E, N * L), s1["offer"],
                              self._replace_index(self.mem_off))
            self._optimize()
        self.cur = 1 - self.cur
        return done

    def episode(self):
        """One episode (env.reset() only gathers observations, SchedulingEnvironment.py:85-109)."""
        while not self.step_round():
            pass
        if self.episodes % self.hp.target_update == 0 and not self.hp.random_policy:
            self.acc.sync_target()
            self.off.sync_target()
        self.episodes += 1

    def flags(self) -> int:
        return self.env.flags()
