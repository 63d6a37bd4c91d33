"""Batched PPO training loop over E env replicas (the trainPPO.py loop, trainPPO.py:133-227).

One ``iteration`` = UPDATE_STEP rounds of (policy act -> env step -> buffer
writes) followed by the PPO update of every unit type, the cadence of
``trainPPO.py:169`` (update when ``world.round % UPDATE_STEP == 0``).
Everything stays on the device: observations are written by the env kernel
straight into the rollout buffers, actions/log-probs by the act kernel.

Architectures (SchedulingEnvironment.py:253-348):
  ``divided`` — PPODividedFixedPriceEnv / PPODividedFreePriceEnv: one net per unit,
  ``local``   — LocallySharedParamsDividedFixedPriceEnv (+ the free-price variant
                BASELINE cfg3 names): one net per agent and unit type,
                CENTRALISATION_SAMPLE sub-units drawn per agent (Agent.py:708-728),
  ``global``  — GloballySharedParamsDividedFixedPriceEnv: one net per unit type,
                CENTRALISATION_SAMPLE (agent, sub-unit) pairs (SchedulingEnvironment.py:314-329).

Multi-GPU: replicas shard across ranks (weak scaling); the nets are shared, so
each optimizer step all-reduces one flattened gradient buffer (RCCL).
"""
from __future__ import annotations

import ctypes as ct
import os
import random
import time
import warnings
from dataclasses import dataclass, field

import numpy as np
import torch

from . import abi
from ._lib import ABI_LOADED, hip_capture, ptr
from .env import BatchedEnv
from .ppo import (ActFrag, PPOGroup, PriceTable, act_round_free, combine_losses, discounted_returns, offer_act_free,
                  reference_init_order, reference_nets, unit_returns)


@dataclass
class Hyper:
    """RL hyper-parameters of trainPPO.py:66-84 (defaults: trainPPO.py)."""
    lr_actor: float = 0.003
    lr_critic: float = 0.01
    eps_clip: float = 0.2
    acceptor_gamma: float | None = None   # default -((1-maxLen)/maxLen) + 0.04 (trainPPO.py:72)
    offer_gamma: float = 0.5
    raw_k_epochs: int = 3
    centralisation_sample: int = 2
    update_step: int = 200
    extra: dict = field(default_factory=dict)


def _k_epochs(raw, factor):
    return max(round(raw / factor), 1)  # trainPPO.py:76-77 (Python round: half-even)


class _Unit:
    """Rollout buffers + PPO group of one unit type (acceptor / offer / price chooser)."""

    def __init__(self, name, E, T, n_units, per_group, in_dim, stride, n_actions, group: PPOGroup, device,
                 reward_dtype, unit_major: bool = False):
        self.name, self.E, self.T, self.U, self.S = name, E, T, n_units, per_group
        self.D, self.stride = in_dim, stride
        self.group = group
        # unit_major: actions / log-probs stored [U][T][E] (one unit's rows of every replica are
        # contiguous for the update's gathers); .actions / .logprobs stay [T][E][U] views
        self.unit_major = unit_major
        if unit_major:
            self.actions_um = torch.zeros((n_units, T, E), dtype=torch.int8, device=device)
            self.logprobs_um = torch.zeros((n_units, T, E), dtype=torch.float32, device=device)
            self.actions = self.actions_um.permute(1, 2, 0)
            self.logprobs = self.logprobs_um.permute(1, 2, 0)
        else:
            self.actions = torch.zeros((T, E, n_units), dtype=torch.int8, device=device)
            self.logprobs = torch.zeros((T, E, n_units), dtype=torch.float32, device=device)
        self.rewards = torch.zeros((T, E, n_units), dtype=reward_dtype, device=device)

    def batch(self, states_i8, u_sel):
        """Gather the update batch of the selected unit per group (u_sel [G] long)."""
        T, E, G = self.T, self.E, u_sel.numel()
        x = states_i8.index_select(2, u_sel)[..., : self.D]               # [T, E, G, D]
        x = x.permute(2, 0, 1, 3).reshape(G, T * E, self.D).float()
        a = self.actions.index_select(2, u_sel).permute(2, 0, 1).reshape(G, T * E).long()
        lp = self.logprobs.index_select(2, u_sel).permute(2, 0, 1).reshape(G, T * E)
        r = self.rewards.index_select(2, u_sel).float().reshape(T, E * G)
        ret = discounted_returns(r, self.group.gamma)                     # [E*G, T]
        ret = ret.view(E, G, T).permute(1, 2, 0).reshape(G, T * E)
        return x, a, lp, ret


def env_seed(seed: int, rank: int, n_envs: int) -> int:
    """Base seed of a rank's replicas: replica e of rank r is random.seed(base + e), so the ranks'
    job streams are disjoint for seeds up to 1000003 / world_size apart."""
    return seed * 1_000_003 + rank * n_envs


def allreduce_mean_grads(params, world_size: int, group=None):
    """Average the gradients over ranks with one flattened all-reduce (RCCL over xGMI on GPUs,
    gloo on CPU). Shards are equal, so the mean of the per-rank mean losses' gradients is the
    gradient of the mean over all replicas."""
    import torch.distributed as dist
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch._utils._flatten_dense_tensors(grads)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.div_(world_size)
    for g, f in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
        g.copy_(f)


def broadcast_params(groups, group=None):
    """Rank 0's weights to every rank (identical start), then policy_old <- policy."""
    import torch.distributed as dist
    for grp in groups:
        for p in grp.policy.parameters():
            dist.broadcast(p.data, src=0, group=group)
        grp.sync_old()


class EnvParts:
    """The rank's E replicas as P contiguous parts [e0, e1), each its own BatchedEnv (replica e keeps
    random.seed(base + e) whatever the split). One part per rollout stream (Trainer.round)."""

    def __init__(self, cfg, E: int, base_seed: int, n_parts: int, device):
        assert E % n_parts == 0
        w = E // n_parts
        self.parts = [(BatchedEnv(cfg, w, seed=base_seed + k * w, device=device), k * w, (k + 1) * w)
                      for k in range(n_parts)]
        self.E = E
        self.shape = self.parts[0][0].shape

    @property
    def round(self) -> int:
        return self.parts[0][0].round

    def flags(self) -> int:
        f = 0
        for env, _, _ in self.parts:
            f |= env.flags()
        return f


class Trainer:
    def __init__(self, cfg: abi.MsConfig, n_envs: int, arch: str = "local", hyper: Hyper | None = None, seed: int = 0,
                 device=None, rank: int = 0, world_size: int = 1, process_group=None, fused: bool = True,
                 use_graph: bool = True, common_rows: bool = True, rollout_streams: int = 1, metrics: bool = False,
                 episode_length: int | None = None, compact: bool = True):
        assert arch in ("divided", "local", "global")
        self.fused = fused  # fused HIP gradient (ms_ppo_grad) vs torch autograd
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        torch.cuda.set_device(self.device)
        self.hp = hyper or Hyper()
        if episode_length is not None:  # episodeLength (world.py:243): the env's `done` cadence
            cfg = abi.MsConfig.from_buffer_copy(cfg)
            cfg.episode_length = int(episode_length)
        self.cfg, self.arch, self.E = cfg, arch, int(n_envs)
        self.rank, self.world_size, self.pg = rank, world_size, process_group
        self.seed = seed
        # rollout_streams > 1: the replicas split into that many parts, each stepped on its own HIP
        # stream, so one part's env round (latency-bound) runs beside another part's act kernels
        # (VALU-bound); the parts share the rollout rings and the nets
        assert rollout_streams >= 1 and self.E % rollout_streams == 0
        self.env = EnvParts(cfg, self.E, env_seed(seed, rank, self.E), rollout_streams, self.device)
        self.streams = [None] + [torch.cuda.Stream(device=self.device) for _ in range(rollout_streams - 1)]
        s = self.env.shape
        N, C, L = s.n_agents, s.n_cores, s.collection_length
        self.N, self.C, self.L = N, C, L
        self.free = bool(cfg.free_prices)
        T = self.T = self.hp.update_step
        hp = self.hp
        max_len = max(cfg.job_length[: cfg.n_kinds])
        acc_gamma = hp.acceptor_gamma if hp.acceptor_gamma is not None else -((1 - max_len) / max_len) + 0.04
        # K epochs and groups per architecture (trainPPO.py:54-55,76-77; PPOmodules.py:289,304)
        if arch == "divided":
            ga, go, k_acc, k_off = N * C, N * L, _k_epochs(hp.raw_k_epochs, 1), _k_epochs(hp.raw_k_epochs, 1)
            if self.free:
                k_off = hp.raw_k_epochs  # FreePriceOfferPPO uses env.RAW_K_EPOCHS
        elif arch == "local":
            ga, go, k_acc, k_off = N, N, _k_epochs(hp.raw_k_epochs, C), _k_epochs(hp.raw_k_epochs, L)
        else:
            ga, go, k_acc, k_off = 1, 1, _k_epochs(hp.raw_k_epochs, N * C), _k_epochs(hp.raw_k_epochs, N * L)
        self.k_acc, self.k_off = k_acc, k_off
        allreduce = self._allreduce if world_size > 1 else None
        # initial weights: the reference's construction order on torch's CPU generator, so a seeded
        # Trainer starts from the weights the reference's agents would draw (same on every rank)
        torch.manual_seed(seed)
        dims = dict(acc=(s.acc_obs_dim, s.acc_actions), off=(s.off_obs_dim, s.off_actions), price=(4, s.price_actions))
        order = reference_init_order(arch, N, C, L, self.free)
        nets = reference_nets(order, {k: dims[k] for k in set(order)})
        dev = self.device
        mk = lambda G, D, A, gamma, K, init: PPOGroup(G, D, A, hp.lr_actor, hp.lr_critic, gamma, hp.eps_clip, K, dev,
                                                      allreduce, init_nets=init)
        self.acc = _Unit("acceptor", self.E, T, N * C, (N * C) // ga, s.acc_obs_dim, s.acc_obs_stride, s.acc_actions,
                         mk(ga, s.acc_obs_dim, s.acc_actions, acc_gamma, k_acc, nets["acc"]), dev, torch.int32)
        self.off = _Unit("offer", self.E, T, N * L, (N * L) // go, s.off_obs_dim, s.off_obs_stride, s.off_actions,
                         mk(go, s.off_obs_dim, s.off_actions, hp.offer_gamma, k_off, nets["off"]), dev, torch.float32)
        self.price = None
        if self.free:
            # MS_PRICE_UNIT_MAJOR=1: the price chooser's rollout rows unit-major, so its update (keyed
            # rows) gathers one unit's rows of every replica contiguously instead of 4 B of every 256 B
            # [E][U] line. Measured at cfg3: k_key_gather 344 -> 279 us, but the act launch's scattered
            # price writes +1.3 us per round: no net gain, so off by default
            self.price_unit_major = os.environ.get("MS_PRICE_UNIT_MAJOR", "0") == "1"
            self.price = _Unit("price", self.E, T, N * L, (N * L) // go, 4, 4, s.price_actions,
                               mk(go, 4, s.price_actions, hp.offer_gamma, k_off, nets["price"]), dev, torch.float32,
                               unit_major=self.price_unit_major)
        if self.free and os.environ.get("MS_PRICE_KEYED", "1") == "0":
            self.price.group.row_keys = 1  # the price chooser's gradient on the tile path (A/B measurements)
        if world_size > 1:
            self._broadcast_params()
        # A single net's item i takes word (i >> 6) & 1 of the draw countered by item i & ~64 (k_act_common's rule on
        # the call's group item index e * S + s), so a shard or part draws what one call over all replicas would
        # only when its first group item, (rank * E + e0) * S, is a multiple of 128. Otherwise the
        # streams stay independent but a split run no longer reproduces the unsplit one: say so.
        if world_size > 1 or rollout_streams > 1:
            per_group = [("acceptor", self.acc.S)] + ([] if self.free else [("offer", self.off.S)])
            for _, e0, _ in self.env.parts:
                for name, S in per_group:
                    if ((rank * self.E + e0) * S) % 128:
                        warnings.warn("%s draws of replicas from %d differ from an unsplit run's: (rank * E + e0) * %d "
                                      "is not a multiple of 128" % (name, rank * self.E + e0, S))
        # observation ring: slot t holds the state acted on at round t; slot T the next state. With
        # compact (and common_rows) the acceptor observations are kept as the env emits them
        # compactly: the owner row of every core + the owners (C rows per replica instead of N*C;
        # Agent.py:167-212), which the act and gradient kernels read directly
        self.compact = bool(compact and common_rows and s.acc_obs_stride >= 16)  # the common-row kernels' range
        if self.compact:
            self.acc_rows = torch.zeros((T + 1, self.E, C, s.acc_obs_stride), dtype=torch.int8, device=dev)
            self.acc_owner = torch.zeros((T + 1, self.E, C), dtype=torch.int8, device=dev)
            self.acc_obs = None
        else:
            self.acc_obs = torch.zeros((T + 1, self.E, N * C, s.acc_obs_stride), dtype=torch.int8, device=dev)
        self.off_obs = torch.zeros((T + 1, self.E, N * L, s.off_obs_stride), dtype=torch.int8, device=dev)
        # price chooser inputs [T][E][U][4] (unit-major: stored [U][T][E][4], self.price_obs its view)
        self.price_obs_um = None
        if self.free and self.price_unit_major:
            self.price_obs_um = torch.zeros((N * L, T, self.E, 4), dtype=torch.int8, device=dev)
            self.price_obs = self.price_obs_um.permute(1, 2, 0, 3)
        else:
            self.price_obs = torch.zeros((T, self.E, N * L, 4), dtype=torch.int8, device=dev) if self.free else None
        self.env_price = torch.zeros((self.E, N * L), dtype=torch.int8, device=dev)
        # the price chooser samples from a table of its few possible inputs, rebuilt from the current
        # weights at the start of every rollout (PriceTable; bit-identical to computing the net)
        self.price_table = PriceTable(cfg, self.price.group.policy_old) if (self.free and self.compact) else None
        # the acceptor row of a core the agent does not own (Agent.py:167-212): most acceptor rows
        # equal it, and the act / gradient kernels compute its network output once
        self.common_rows = common_rows
        O = s.max_offers
        crow = [0, -1, -1] + [-2] * (2 * O) + [0] * (s.acc_obs_stride - s.acc_obs_dim)
        self.acc_common = torch.tensor(crow, dtype=torch.int8, device=dev)
        # the acting nets' weight fragments (and the acceptors' common-row table), rebuilt at the start
        # of every rollout like the price table (ActFrag; bit-identical to acting without them)
        # (MS_ACT_FRAG=0: without them, for A/B measurements)
        use_frag = os.environ.get("MS_ACT_FRAG", "1") != "0"
        self.off_frag = ActFrag(self.off.group.policy_old, s.off_obs_stride) if use_frag else None
        self.acc_frag = ActFrag(self.acc.group.policy_old, s.acc_obs_stride, self.acc_common) if use_frag else None
        self.agent_reward = torch.zeros((self.E, N), dtype=torch.int32, device=dev)
        self.auct_reward = torch.zeros((self.E, C), dtype=torch.int32, device=dev)
        self.rng = random.Random(seed)  # sub-unit draws (random.randint), identical on every rank
        self.rng_ctr = torch.zeros(1, dtype=torch.int64, device=dev)  # device Philox offset base
        self.use_graph = use_graph
        self.graph = None
        self.rounds_done = 0
        self._policy_version = 0  # bumped by update(); the acting tables record the version they saw
        self.iterations = 0
        for env, e0, e1 in self.env.parts:
            env.reset(dict(self._acc_out(0, e0, e1), offer=self.off_obs[0][e0:e1]))
        # episode metrics (trainPPO.py:153-226): the env kernel adds every round into per-replica
        # accumulators, slot (round // episodeLength) % slots; finished episodes are read after each
        # rollout (metrics.py) and their slots zeroed before reuse
        self.ep_len = int(self.cfg.episode_length)
        self.metric_slots = -(-T // self.ep_len) + 1
        self.metric_bufs = [env.metrics_buffer(self.metric_slots) for env, _, _ in self.env.parts] if metrics else None
        self.episode_log = []
        # one rank: each unit type's update on its own stream (MS_UPDATE_STREAMS=0: one stream). Round 4: the
        # update 10.06 -> 9.63 ms but the next rollout 14.50 -> 15.63 ms (every rollout launch slower after a
        # multi-stream update graph), so it was off. Round 6, with cfg3's rollout one launch: update 8.50 -> 8.05 ms,
        # rollout 9.99 -> 10.11 ms, iteration 18.50 -> 18.18 ms (profiles/r7b), so it is on
        self.update_streams = os.environ.get("MS_UPDATE_STREAMS", "1") == "1"
        # fixed-price rounds with one net per role (cfg2): round t's env launch also samples round t + 1's
        # actions from the observations it just built (ms_env_step_act), so a round is one launch
        # (MS_ENV_FUSED_ACT=0: the act launch and the env launch of every round, for A/B measurements)
        # (T > 1: the fused acting writes round t + 1's ring slots)
        self.fused_step = (self.compact and not self.free and self.acc.group.policy.G == 1 and
                           self.off.group.policy.G == 1 and self.acc_frag is not None and self.T > 1 and
                           os.environ.get("MS_ENV_FUSED_ACT", "1") != "0" and self.metric_bufs is None and
                           all(env.fused_act_supported() for env, _, _ in self.env.parts))
        # ... and the whole rollout's rounds are one launch (ms_env_rollout_act): each wave steps and acts
        # for its replicas round after round (MS_ENV_ROLLOUT=0: one launch per round, for A/B measurements)
        self.fused_rollout = self.fused_step and os.environ.get("MS_ENV_ROLLOUT", "1") != "0"
        # locally shared free-price rounds (cfg3): the whole rollout in one launch too (ms_env_rollout_act_free):
        # a workgroup steps its replicas, then acts for them with one wave per agent, round after round
        # (MS_ENV_ROLLOUT_FREE=0: an act launch and an env launch per round, for A/B measurements)
        self.fused_rollout_free = (self.compact and self.free and arch == "local" and self.price_table is not None and
                                   self.off_frag is not None and not self.price_unit_major and self.T > 1 and
                                   self.metric_bufs is None and os.environ.get("MS_ENV_ROLLOUT_FREE", "1") != "0" and
                                   all(env.rollout_free_supported() for env, _, _ in self.env.parts))
        # ... and its acceptor items of cores their agent does not own (sampled from the common row's table; the env
        # reads only the owner's acceptor action) are left to a second kernel (ms_env_rollout_fill_common) after the
        # launch. MS_DEFER_COMMON=1: iteration() runs it inside the update instead, on the acceptor's stream beside
        # the offer and price gradients (offsets from a snapshot of rng_ctr taken by the rollout); measured even
        # (17.84-17.92 ms per iteration either way, profiles/r7: the update is as throughput-bound as the rollout)
        self.defer_common = (self.fused_rollout_free and self.update_streams and self.world_size == 1 and self.fused and
                             os.environ.get("MS_DEFER_COMMON", "0") == "1")
        self.rng_snap = torch.zeros(1, dtype=torch.int64, device=self.device)
        # the rollout's owned acceptor items by core ([T][E][C]; ABI 18): the fill then writes the acceptor rings'
        # rows whole (MS_FILL_OWN=0: the rollout writes them into the rings, one item in eight of a line)
        self.acc_own = None
        if self.fused_rollout_free and ABI_LOADED >= 18 and os.environ.get("MS_FILL_OWN", "1") != "0":
            self.acc_own = (torch.zeros((T, self.E, C), dtype=torch.int8, device=dev),
                            torch.zeros((T, self.E, C), dtype=torch.float32, device=dev))
        self._fill_args = []
        self.span_every = 0  # > 0: every span_every-th round's env launches record their span (bench)
        self.spans = None
        self.timings = dict(rollout=0.0, update=0.0)

    @classmethod
    def from_named(cls, name: str, n_envs=None, update_step=200, seed=0, device=None, **kw):
        cfg = abi.named_config(name)
        arch = {"cfg1": "divided", "cfg2": "global", "cfg3": "local", "cfg4": "divided", "cfg5": "divided"}[name]
        hp = Hyper(update_step=update_step)
        if name == "cfg3":  # trainPPOExperiment4.py:96-98 (free prices): RAW_K 2, ACCEPTOR_GAMMA 0.95
            hp.raw_k_epochs = 2
            hp.acceptor_gamma = -((1 - 5) / 5) + 0.15
        return cls(cfg, n_envs or abi.NAMED_ENVS[name], arch=kw.pop("arch", arch), hyper=hp, seed=seed, device=device,
                   **kw)

    def _acc_out(self, t, e0, e1):
        """The env's acceptor observation outputs for ring slot t, replicas [e0, e1)."""
        if self.compact:
            return dict(core_rows=self.acc_rows[t][e0:e1], core_owner=self.acc_owner[t][e0:e1])
        return dict(acceptor=self.acc_obs[t][e0:e1])

    def acceptor_rows(self, t0: int = 0, t1: int | None = None):
        """The [t1 - t0, E, N*C, stride] acceptor rows of ring slots t0..t1-1 (regenerated from the
        compact form when the ring is compact)."""
        t1 = self.T + 1 if t1 is None else t1
        if not self.compact:
            return self.acc_obs[t0:t1]
        from .ppo import regen_acceptor_rows
        return regen_acceptor_rows(self.acc_rows[t0:t1], self.acc_owner[t0:t1], self.acc_common, self.N)

    # ---- distributed helpers
    def _allreduce(self, params):
        allreduce_mean_grads(params, self.world_size, self.pg)

    def _broadcast_params(self):
        broadcast_params([u.group for u in self.units()], self.pg)

    def units(self):
        return [u for u in (self.acc, self.off, self.price) if u is not None]

    # ---- rollout
    def _prepare_acting(self):
        """The acting kernels' per-rollout tables from policy_old: the price chooser's table of its
        possible inputs and the act weight fragments (ms_act_prepare). They are rebuilt at the start
        of every rollout (inside the rollout graph) and by round() after an update changed
        policy_old (sync_old bumps _policy_version)."""
        if self.price_table is not None:
            self.price_table.build(self.price.group.policy_old)
        if self.off_frag is not None:
            self.off_frag.build(self.off.group.policy_old)
            self.acc_frag.build(self.acc.group.policy_old)
        self._acting_version = self._policy_version

    def round(self, t: int):
        """getActionForAllAgents + env.step + saveRewards for round t of the iteration
        (trainPPO.py:160-167), part by part: part k's launches go to stream k."""
        if getattr(self, "_acting_version", -1) != self._policy_version:
            self._prepare_acting()
        for k in range(len(self.env.parts)):
            self._round_part(t, k)

    def _round_part(self, t: int, k: int):
        self._act_part(t, k)
        self._step_part(t, k)

    def _act_part(self, t: int, k: int):
        """getActionForAllAgents of round t for replica part k (on stream k)."""
        if self.fused_step and t > 0:
            return  # sampled by round t - 1's env launch (_step_part)
        env, e0, e1 = self.env.parts[k]
        st = self.streams[k]
        E, N, C, L = e1 - e0, self.N, self.C, self.L
        # one Philox key for every rank and part; the counter's row is global (replica_base = this
        # part's first replica in the whole job, rank-major), so a replica draws the same numbers on
        # any number of ranks or parts (when rank * E * units per group is a multiple of 128, ms_mlp_params)
        # offsets: static per round + the device counter (advanced per rollout)
        seed = self.seed * 7919
        rb = self.rank * self.E + e0
        base = 8 * t
        sl = lambda x: x[e0:e1]
        # per agent: offer units then acceptors (Agent.py:504-515); separate streams per unit type
        if self.free:
            # FreePriceOfferPPO.selectAction (PPOmodules.py:312-332): core chooser, then the price
            # chooser on [obs[2a:2a+2], obs[-2:]] or the dummy [-5,-5,-5,-5] when a == 0, one launch
            out = dict(core_action=sl(self.off.actions[t]), core_logprob=sl(self.off.logprobs[t]),
                       price_state=sl(self.price_obs[t]), price_action=sl(self.price.actions[t]),
                       price_logprob=sl(self.price.logprobs[t]), env_price=sl(self.env_price))
            pus = 0
            if self.price_unit_major:  # [U][E'] views of the [U][T][E] rings, units T*E rows apart
                out.update(price_state=self.price_obs_um[:, t, e0:e1], price_action=self.price.actions_um[:, t, e0:e1],
                           price_logprob=self.price.logprobs_um[:, t, e0:e1])
                pus = self.T * self.E
            if self.compact:  # the acceptors too, in the same launch
                act_round_free(self.off.group.policy_old, self.price.group.policy_old, sl(self.off_obs[t]),
                               self.acc.group.policy_old, sl(self.acc_rows[t]), sl(self.acc_owner[t]), self.acc_common,
                               C, seed, base + 1, base + 3, out, sl(self.acc.actions[t]), sl(self.acc.logprobs[t]),
                               offset_dev=self.rng_ctr, stream=st, price_table=self.price_table,
                               price_unit_stride=pus, core_frag=self.off_frag, acc_frag=self.acc_frag,
                               replica_base=rb)
            else:
                offer_act_free(self.off.group.policy_old, self.price.group.policy_old, sl(self.off_obs[t]), C, seed,
                               base + 1, out, offset_dev=self.rng_ctr, stream=st, price_unit_stride=pus,
                               core_frag=self.off_frag, replica_base=rb)
        elif self.compact and ABI_LOADED < 16:
            # (an older A/B library: no fixed-price act_round_free; the two launches)
            self.off.group.policy_old.act(sl(self.off_obs[t]), N * L, seed, base + 1, action=sl(self.off.actions[t]),
                                          logprob=sl(self.off.logprobs[t]), offset_dev=self.rng_ctr, stream=st,
                                          frag=self.off_frag, replica_base=rb)
            self.acc.group.policy_old.act_compact(sl(self.acc_rows[t]), sl(self.acc_owner[t]), N * C, seed, base + 3,
                                                  self.acc_common, action=sl(self.acc.actions[t]),
                                                  logprob=sl(self.acc.logprobs[t]), stream=st, offset_dev=self.rng_ctr,
                                                  frag=self.acc_frag, replica_base=rb)
        elif self.compact:
            # a fixed-price round: the offer units and the compact acceptors in one launch
            act_round_free(self.off.group.policy_old, None, sl(self.off_obs[t]), self.acc.group.policy_old,
                           sl(self.acc_rows[t]), sl(self.acc_owner[t]), self.acc_common, C, seed, base + 1, base + 3,
                           dict(core_action=sl(self.off.actions[t]), core_logprob=sl(self.off.logprobs[t])),
                           sl(self.acc.actions[t]), sl(self.acc.logprobs[t]), offset_dev=self.rng_ctr, stream=st,
                           core_frag=self.off_frag, acc_frag=self.acc_frag, replica_base=rb)
        else:
            self.off.group.policy_old.act(sl(self.off_obs[t]), N * L, seed, base + 1, action=sl(self.off.actions[t]),
                                          logprob=sl(self.off.logprobs[t]), offset_dev=self.rng_ctr, stream=st,
                                          frag=self.off_frag, replica_base=rb)
        if not self.compact:  # (compact acceptors acted above, in the offers' launch)
            self.acc.group.policy_old.act(sl(self.acc_obs[t]), N * C, seed, base + 3, action=sl(self.acc.actions[t]),
                                          logprob=sl(self.acc.logprobs[t]), offset_dev=self.rng_ctr,
                                          common_row=self.acc_common if self.common_rows else None, stream=st,
                                          frag=self.acc_frag, replica_base=rb)

    def _step_part(self, t: int, k: int):
        """env.step + saveRewards of round t for replica part k (on stream k)."""
        env, e0, e1 = self.env.parts[k]
        st = self.streams[k]
        E, N, C, L = e1 - e0, self.N, self.C, self.L
        sl = lambda x: x[e0:e1]
        obs = dict(self._acc_out(t + 1, e0, e1), offer=sl(self.off_obs[t + 1]))
        rew = dict(offer=sl(self.off.rewards[t]).view(E, N, L), acceptor=sl(self.acc.rewards[t]).view(E, N, C),
                   agent=sl(self.agent_reward), auctioneer=sl(self.auct_reward),
                   price=sl(self.price.rewards[t]).view(E, N, L) if self.free else None)
        ev = dict(launch_span=self.spans[t // self.span_every, k]) if self.span_every and t % self.span_every == 0 else None
        if self.metric_bufs is not None:
            ev = dict(ev or {}, metrics=self.metric_bufs[k])
        nxt = self._fused_next(t + 1, k) if self.fused_step and t + 1 < self.T else None
        env.step(sl(self.acc.actions[t]).view(E, N, C), sl(self.off.actions[t]).view(E, N, L),
                 sl(self.env_price).view(E, N, L) if self.free else None, obs=obs, rewards=rew, events=ev, stream=st,
                 next_act=nxt)

    def _fused_next(self, t: int, k: int):
        """Round t's getActionForAllAgents (the fixed-price pair of _act_part) for replica part k, as the
        acting fused into round t - 1's env launch."""
        e0, e1 = self.env.parts[k][1:]
        sl = lambda x: x[e0:e1]
        N, C, L = self.N, self.C, self.L
        seed, base, rb = self.seed * 7919, 8 * t, self.rank * self.E + e0
        return abi.MsFusedAct(self.off.group.policy_old.mlp_params(self.off_frag, rb * N * L),
                              self.acc.group.policy_old.mlp_params(self.acc_frag, rb * N * C), ptr(self.acc_common),
                              seed, base + 1, base + 3, ptr(self.rng_ctr), ptr(sl(self.off.actions[t])),
                              ptr(sl(self.off.logprobs[t])), ptr(sl(self.acc.actions[t])), ptr(sl(self.acc.logprobs[t])))

    def _rollout_part(self, k: int):
        """Rounds 0..T-1 of replica part k (env.step + saveRewards, and the acting of rounds 1..T-1) in
        one launch (ms_env_rollout_act); round 0's acting ran before it (_act_part)."""
        env, e0, e1 = self.env.parts[k]
        E, N, C, L = e1 - e0, self.N, self.C, self.L
        sl = lambda x: x[e0:e1]
        obs = dict(self._acc_out(1, e0, e1), offer=sl(self.off_obs[1]))
        rew = dict(offer=sl(self.off.rewards[0]).view(E, N, L), acceptor=sl(self.acc.rewards[0]).view(E, N, C),
                   agent=sl(self.agent_reward), auctioneer=sl(self.auct_reward))
        ev = dict(launch_span=self.spans[0, k]) if self.span_every else None
        b = lambda x: x.stride(0) * x.element_size()  # bytes between ring slots t and t + 1
        strides = abi.MsRoundStrides(b(self.acc.actions), b(self.off.actions), b(self.acc_rows), b(self.acc_owner),
                                     b(self.off_obs), b(self.off.rewards), b(self.acc.rewards), 0, 0,
                                     b(self.off.actions), b(self.off.logprobs), b(self.acc.actions),
                                     b(self.acc.logprobs), 8)
        env.rollout_act(sl(self.acc.actions[0]).view(E, N, C), sl(self.off.actions[0]).view(E, N, L), obs, rew,
                        self._fused_next(1, k), strides, self.T, act_after_last=False, events=ev,
                        stream=self.streams[k])

    def _fused_next_free(self, t: int, k: int):
        """Round t's acting of a locally shared free-price round (act_round_free of _act_part) for replica part k,
        fused into round t - 1 of the one-launch rollout: (abi.MsFusedActFree, its output tensors)."""
        e0, e1 = self.env.parts[k][1:]
        sl = lambda x: x[e0:e1]
        N, C, L = self.N, self.C, self.L
        seed, base, rb = self.seed * 7919, 8 * t, self.rank * self.E + e0
        out = dict(core_action=sl(self.off.actions[t]), core_logprob=sl(self.off.logprobs[t]),
                   price_state=sl(self.price_obs[t]), price_action=sl(self.price.actions[t]),
                   price_logprob=sl(self.price.logprobs[t]), env_price=sl(self.env_price),
                   acc_action=sl(self.acc.actions[t]), acc_logprob=sl(self.acc.logprobs[t]))
        names = ("core_action", "core_logprob", "price_state", "price_action", "price_logprob", "env_price",
                 "acc_action", "acc_logprob")
        nxt = abi.MsFusedActFree(self.off.group.policy_old.mlp_params(self.off_frag, rb * N * L),
                                 self.price.group.policy_old.mlp_params(),
                                 self.acc.group.policy_old.mlp_params(self.acc_frag, rb * N * C), ptr(self.acc_common),
                                 ct.addressof(self.price_table.struct), seed, base + 1, base + 3, ptr(self.rng_ctr),
                                 *[ptr(out[n]) for n in names])
        if self.acc_own is not None:
            out.update(own_action=sl(self.acc_own[0][t]), own_logprob=sl(self.acc_own[1][t]))
            nxt.own_action, nxt.own_logprob = ptr(out["own_action"]), ptr(out["own_logprob"])
        return nxt, out

    def _rollout_part_free(self, k: int):
        """Rounds 0..T-1 of replica part k of a locally shared free-price rollout (env.step + saveRewards, and the
        acting of rounds 1..T-1) in one launch (ms_env_rollout_act_free); round 0's acting ran before it."""
        env, e0, e1 = self.env.parts[k]
        E, N, C, L = e1 - e0, self.N, self.C, self.L
        sl = lambda x: x[e0:e1]
        obs = dict(self._acc_out(1, e0, e1), offer=sl(self.off_obs[1]))
        rew = dict(offer=sl(self.off.rewards[0]).view(E, N, L), acceptor=sl(self.acc.rewards[0]).view(E, N, C),
                   agent=sl(self.agent_reward), auctioneer=sl(self.auct_reward),
                   price=sl(self.price.rewards[0]).view(E, N, L))
        ev = dict(launch_span=self.spans[0, k]) if self.span_every else None
        b = lambda x: x.stride(0) * x.element_size()  # bytes between ring slots t and t + 1
        strides = abi.MsRoundStridesFree(b(self.acc.actions), b(self.off.actions), b(self.acc_rows), b(self.acc_owner),
                                         b(self.off_obs), b(self.off.rewards), b(self.price.rewards),
                                         b(self.acc.rewards), 0, 0, b(self.off.actions), b(self.off.logprobs),
                                         b(self.price_obs), b(self.price.actions), b(self.price.logprobs),
                                         b(self.acc.actions), b(self.acc.logprobs), 8)
        if self.acc_own is not None:
            strides.next_own_action, strides.next_own_logprob = b(self.acc_own[0]), b(self.acc_own[1])
        nxt, out = self._fused_next_free(1, k)
        nxt.defer_common = int(self.defer_common)
        env.rollout_act_free(sl(self.acc.actions[0]).view(E, N, C), sl(self.off.actions[0]).view(E, N, L), obs, rew,
                             nxt, out, strides, self.T, act_after_last=False, events=ev, stream=self.streams[k])
        if self.defer_common:  # the fill's arguments: the same call with the offsets of this rollout (snapshot)
            fill = abi.MsFusedActFree.from_buffer_copy(nxt)
            fill.offset_dev = ptr(self.rng_snap)
            self._fill_args.append((env, obs, fill, strides))

    def fill_common(self, stream=None):
        """The deferred acceptor items of the last one-launch rollout (defer_common; idempotent)."""
        for env, obs, fill, strides in self._fill_args:
            env.fill_common(obs, fill, strides, self.T, act_after_last=False, stream=stream)

    def record_launch_spans(self, every: int):
        """Every `every`-th round's env launches record their span (first wave start, last wave end
        on the 100 MHz s_memrealtime clock, and each wave's shader-clock cycles) into self.spans
        [ceil(T / every)][parts][waves][4]; read with launch_spans_us() / launch_clock_mhz(). Set before the first
        rollout (the HIP graph captures it)."""
        self.span_every = int(every)
        w = self.env.parts[0][2] - self.env.parts[0][1]
        n = -(-self.T // self.span_every)  # row t // every holds round t's launches (t % every == 0)
        self.spans = torch.zeros((n, len(self.env.parts), w, 4), dtype=torch.int64, device=self.device)

    def sampled_spans(self):
        """The recorded rounds' spans ([ceil(T / span_every)][parts][waves][4], contiguous)."""
        return self.spans

    def launch_spans_us(self, sampled=None):
        """Durations (us) of the recorded env launches of the last rollout (fused_rollout: the one
        launch of each part over T, per round), or of `sampled` (a copy of sampled_spans())."""
        sp = (self.sampled_spans() if sampled is None else sampled).cpu().numpy()  # [rounds][parts][waves][4]
        if self.fused_rollout or self.fused_rollout_free:
            out = []
            for w in sp[0]:  # [parts][waves][4]: round 0's slot holds the launch
                w = w[w[:, 1] > 0]
                out.append(float(w[:, 1].max() - w[:, 0].min()) / 100.0 / self.T)
            return out
        out = []
        for r in range(sp.shape[0]):
            for k in range(sp.shape[1]):
                w = sp[r, k]
                w = w[w[:, 1] > 0]  # the waves of the launch
                out.append(float(w[:, 1].max() - w[:, 0].min()) / 100.0)
        return out

    def launch_clock_mhz(self, sampled=None):
        """Median shader clock (MHz) of the recorded env launches' waves: shader cycles over 100 MHz ticks."""
        sp = (self.sampled_spans() if sampled is None else sampled).cpu().numpy().reshape(-1, 4)
        sp = sp[(sp[:, 1] > sp[:, 0]) & (sp[:, 3] > sp[:, 2])]
        if len(sp) == 0:
            return None
        return float(np.median((sp[:, 3] - sp[:, 2]) / (sp[:, 1] - sp[:, 0]) * 100.0))

    def _rollout_body(self):
        cur = torch.cuda.current_stream(self.device)
        if self.span_every:
            self.spans.zero_()
        self._prepare_acting()
        self._fill_args = []
        if self.defer_common:
            self.rng_snap.copy_(self.rng_ctr)
        for s in self.streams[1:]:  # fork: the side streams start after everything queued so far
            s.wait_stream(cur)
        if self.fused_rollout or self.fused_rollout_free:
            for k in range(len(self.env.parts)):
                self._act_part(0, k)
                (self._rollout_part_free if self.fused_rollout_free else self._rollout_part)(k)
        else:
            for t in range(self.T):
                self.round(t)
        for s in self.streams[1:]:  # join
            cur.wait_stream(s)
        self.rng_ctr.add_(8 * self.T)

    def rollout(self, defer_common: bool = False):
        """UPDATE_STEP rounds. With use_graph the first rollout runs eagerly and is then
        captured once into a HIP graph (every pointer is static); later rollouts replay it.
        defer_common (iteration()): leave the deferred acceptor items (self.defer_common) to the update, which
        samples them on the acceptor's stream; otherwise the rings are complete when this returns."""
        if not self.use_graph:
            self._rollout_body()
        elif self.graph is None:
            self._rollout_body()
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with hip_capture(g):
                self._rollout_body()
            self.graph = g
        else:
            self.graph.replay()
        if self.defer_common and not defer_common:
            self.fill_common()
        self.rounds_done += self.T

    # ---- update
    def _draws(self, device=None):
        """Sub-unit selections, in the reference's random.randint order."""
        N, C, L, CS = self.N, self.C, self.L, self.hp.centralisation_sample
        dev = self.device if device is None else device
        if self.arch == "divided":
            sel = dict(acceptor=[torch.arange(N * C, device=dev)], offer=[torch.arange(N * L, device=dev)])
        elif self.arch == "local":
            acc = [[0] * N for _ in range(CS)]
            off = [[0] * N for _ in range(CS)]
            for a in range(N):  # per agent: acceptor draws then offer draws (Agent.py:716-728)
                for i in range(CS):
                    acc[i][a] = a * C + self.rng.randint(0, C - 1)
                for j in range(CS):
                    off[j][a] = a * L + self.rng.randint(0, L - 1)
            sel = dict(acceptor=[torch.tensor(r, device=dev) for r in acc],
                       offer=[torch.tensor(r, device=dev) for r in off])
        else:
            acc, off = [], []
            for _ in range(CS):  # SchedulingEnvironment.py:315-321
                a = self.rng.randint(0, N - 1)
                c = self.rng.randint(0, C - 1)
                acc.append(torch.tensor([a * C + c], device=dev))
            for _ in range(CS):  # SchedulingEnvironment.py:323-329
                a = self.rng.randint(0, N - 1)
                l = self.rng.randint(0, L - 1)
                off.append(torch.tensor([a * L + l], device=dev))
            sel = dict(acceptor=acc, offer=off)
        sel["price"] = sel["offer"]
        return sel

    def update(self):
        """env.updateAgents() (SchedulingEnvironment.py:208-210 / 314-329, Agent.py:524-529,708-728).
        With use_graph the fused update is captured into HIP graphs after its first (eager) run and
        replayed from then on: only this iteration's sub-unit draws are copied to the device
        first. One rank: one graph. Several ranks: one graph per stretch between two gradient
        all-reduces, the RCCL calls eager in between (_capture_update). The returned losses are
        copies of the graph's own tensors."""
        self._policy_version += 1  # policy_old changes: round() rebuilds the acting tables
        if self.use_graph and self.fused:
            return self._update_graphed()
        sel = self._draws()
        if self.fused:
            return self._fused_update({k: torch.cat(v).to(torch.int32) for k, v in sel.items()},
                                      {k: [x.numel() for x in v] for k, v in sel.items()})
        return self._torch_update(sel)

    def _update_rows(self, u):
        """(states, actions, old log-probs) of unit type u for ms_ppo_grad: [T*E, U(, stride)] rows, or
        [U, T*E(, stride)] for a unit-major unit."""
        T, E = self.T, self.E
        if u.unit_major:
            st = self.price_obs_um if u is self.price else None
            return st.reshape(u.U, T * E, u.stride), u.actions_um.reshape(u.U, T * E), u.logprobs_um.reshape(u.U, T * E)
        return (self._states_of(u).reshape(T * E, -1, u.stride), u.actions.view(T * E, u.U),
                u.logprobs.view(T * E, u.U))

    def _states_of(self, u):
        T = self.T
        if u is self.acc:
            return self.acc_rows[:T] if self.compact else self.acc_obs[:T]
        return (self.off_obs if u is self.off else self.price_obs)[:T]

    def _update_graphed(self):
        host = {k: [list(map(int, d.tolist())) for d in v] for k, v in self._draws(device="cpu").items()}
        names = [u.name for u in self.units()]
        flat = [x for k in names for d in host[k] for x in d]
        if getattr(self, "_sel_dev", None) is None:
            self._sel_host = torch.empty(len(flat), dtype=torch.int32, pin_memory=True)
            self._sel_dev = torch.empty(len(flat), dtype=torch.int32, device=self.device)
            self._sel_event = torch.cuda.Event()
            self._sel_counts = {k: [len(d) for d in host[k]] for k in names}
            self.update_graph = None
        self._sel_event.synchronize()  # the previous copy out of the pinned buffer is done
        self._sel_host.copy_(torch.tensor(flat, dtype=torch.int32))
        self._sel_dev.copy_(self._sel_host, non_blocking=True)
        self._sel_event.record()
        views, col = {}, 0
        for k in names:
            n = sum(self._sel_counts[k])
            views[k] = self._sel_dev[col:col + n]
            col += n
        if self.update_graph is None:
            losses = self._fused_update(views, self._sel_counts)  # this iteration's update
            eager_last = {u.name: u.group.last_losses for u in self.units()}
            torch.cuda.synchronize(self.device)
            self._graph_losses = self._capture_update(views)
            self._graph_last = {u.name: list(u.group.last_losses) for u in self.units()}
            for u in self.units():  # the eager run's own losses until the first replay
                u.group.last_losses = eager_last[u.name]
            return losses
        self._replay_update()
        # the graph's loss tensors are overwritten by every replay: hand out copies (G floats per
        # unit type), so losses a caller keeps from earlier iterations stay what they were
        for u in self.units():
            u.group.last_losses = [x.clone() for x in self._graph_last[u.name]]
        return {k: v.clone() for k, v in self._graph_losses.items()}

    def _capture_update(self, views):
        """Capture the fused update: segment i = the kernels between all-reduce i-1 and i (one
        segment on one rank), all in one memory pool. Returns the graph's loss tensors."""
        if self.world_size == 1 and self.update_streams:
            # MS_UPDATE_STREAMS on one rank: the per-unit-type streams are recorded into the graph
            # (fork / join on the capture stream), so replays run the same concurrent form the
            # eager first update ran
            g = torch.cuda.CUDAGraph()
            with hip_capture(g):
                losses = self._fused_update_streams(views, self._sel_counts)
            self.update_graph, self._graph_params = [g], []
            return losses
        out, graphs, params = {}, [], []
        phases = self._fused_phases(views, self._sel_counts, out)
        pool = None
        while True:
            g = torch.cuda.CUDAGraph()
            with hip_capture(g, pool=pool):
                p = next(phases, None)
            if pool is None:
                pool = g.pool()
            graphs.append(g)
            if p is None:
                break
            params.append(p)
        self.update_graph = graphs
        self._graph_params = params
        return out["losses"]

    def _replay_update(self):
        for i, g in enumerate(self.update_graph):
            g.replay()
            if i < len(self._graph_params):
                self._allreduce(self._graph_params[i])

    def _fused_update(self, all_sel, counts):
        """The fused update: all_sel[name] = int32 device [sum of draws' G] sub-units, counts[name]
        = each draw's number of groups."""
        if self.world_size == 1 and self.update_streams:
            return self._fused_update_streams(all_sel, counts)
        out = {}
        for params in self._fused_phases(all_sel, counts, out):
            self._allreduce(params)
        return out["losses"]

    def _fused_phases(self, all_sel, counts, out):
        """_fused_update as a generator: yields the parameters whose gradients the ranks all-reduce
        (several ranks only) and leaves the losses in out["losses"]."""
        T, E = self.T, self.E
        losses = {}
        if self.defer_common:  # the rollout's deferred acceptor items (a trainer switched to several ranks)
            self.fill_common()
        # Each unit type's draws update its nets in sequence (draw d trains on the weights draw d-1
        # left), but the unit types are independent nets: step s of the update = epoch k of draw d
        # of every unit type that has one, with ONE all-reduce of all their gradients (one
        # flattened RCCL call per step) before each type's Adam step.
        steps = {}
        for u in self.units():
            # the returns of every draw's sub-units in one launch: [T][E][sum of G], draw d at
            # column offset d*G (returns depend on the rewards only, not on earlier draws' updates)
            sel_u = all_sel[u.name]
            ret_all = unit_returns(u.rewards, sel_u, u.group.gamma)
            common = self.acc_common if (u is self.acc and self.common_rows) else None
            owner = self.acc_owner[:T].reshape(T * E, self.C) if (u is self.acc and self.compact) else None
            col, seq = 0, []
            rows = self._update_rows(u)
            for n in counts[u.name]:
                ep = u.group.fused_epoch(*rows, ret_all.view(-1)[col:], sel_u[col:col + n], T, E, common_row=common,
                                         returns_ld=sel_u.numel(), core_owner=owner, unit_major=u.unit_major)
                seq += [ep] * u.group.K
                col += n
            steps[u.name] = (u, seq, [])
        # each unit type's loss terms of every (draw, epoch) into one [n][G][3] buffer, combined once at the end
        terms = {name: torch.empty((len(seq), u.group.policy.G, 3), dtype=torch.float32, device=self.device)
                 for name, (u, seq, _) in steps.items()}
        for s in range(max(len(v[1]) for v in steps.values())):
            live = [(u, seq, ls) for u, seq, ls in steps.values() if s < len(seq)]
            for u, seq, ls in live:
                ls.append(seq[s].launch(terms[u.name][s]))
            if self.world_size > 1:
                yield [p for u, _, _ in live for p in u.group.policy.parameters()]
            for u, _, _ in live:
                u.group.hip_optimizer.step()
        for u, _, ls in steps.values():
            losses[u.name] = combine_losses(terms[u.name])
            u.group.last_losses = list(losses[u.name].unbind(0))
            u.group.sync_old()
        self._carry_last_observation()
        out["losses"] = losses

    def _epochs(self, u, sel_u, counts_u):
        """The gradient closures of unit type u's K epochs of every draw, in order."""
        T, E = self.T, self.E
        # the returns of every draw's sub-units in one launch: [T][E][sum of G], draw d at column
        # offset d*G (returns depend on the rewards only, not on earlier draws' updates)
        ret_all = unit_returns(u.rewards, sel_u, u.group.gamma)
        common = self.acc_common if (u is self.acc and self.common_rows) else None
        owner = self.acc_owner[:T].reshape(T * E, self.C) if (u is self.acc and self.compact) else None
        rows = self._update_rows(u)
        col, seq = 0, []
        for n in counts_u:
            ep = u.group.fused_epoch(*rows, ret_all.view(-1)[col:], sel_u[col:col + n], T, E, common_row=common,
                                     returns_ld=sel_u.numel(), core_owner=owner, unit_major=u.unit_major)
            seq += [ep] * u.group.K
            col += n
        return seq

    def _fused_update_streams(self, all_sel, counts):
        """One rank: the unit types' nets are independent, so each type's whole update (its draws'
        epochs, each a gradient then an Adam step) runs on its own stream and the types' gradient
        kernels share the GPU (each is latency-bound at 2-3 waves per SIMD)."""
        cur = torch.cuda.current_stream(self.device)
        units = self.units()
        if getattr(self, "_unit_streams", None) is None:
            self._unit_streams = [torch.cuda.Stream(device=self.device) for _ in units]
        losses = {}
        for st in self._unit_streams:
            st.wait_stream(cur)
        for u, st in zip(units, self._unit_streams):
            with torch.cuda.stream(st):
                if u is self.acc and self.defer_common:
                    self.fill_common(stream=st)  # the rollout's deferred acceptor items, beside the other units
                seq = self._epochs(u, all_sel[u.name], counts[u.name])
                # every (draw, epoch)'s loss terms into one buffer, combined at once (not four small kernels each)
                terms = torch.empty((len(seq), u.group.policy.G, 3), dtype=torch.float32, device=self.device)
                for i, ep in enumerate(seq):
                    ep.launch(terms[i])
                    u.group.hip_optimizer.step(st)
                losses[u.name] = combine_losses(terms)
                u.group.last_losses = list(losses[u.name].unbind(0))
                u.group.sync_old()
        for st in self._unit_streams:
            cur.wait_stream(st)
        self._carry_last_observation()
        return losses

    def _torch_update(self, sel):
        """The torch-autograd update (the numerical reference of the fused one)."""
        T = self.T
        losses = {}
        if self.defer_common:
            self.fill_common()
        for u in self.units():
            ls = []
            st_u = self.acceptor_rows(0, T) if (u is self.acc and self.compact) else self._states_of(u)
            for u_sel in sel[u.name]:
                x, a, lp, ret = u.batch(st_u, u_sel)
                ls += u.group.update(x, a, lp, ret)
            u.group.sync_old()
            losses[u.name] = torch.stack(ls)
        self._carry_last_observation()
        return losses

    def _carry_last_observation(self):
        """The next iteration starts from the last observation."""
        if self.compact:
            self.acc_rows[0].copy_(self.acc_rows[self.T])
            self.acc_owner[0].copy_(self.acc_owner[self.T])
        else:
            self.acc_obs[0].copy_(self.acc_obs[self.T])
        self.off_obs[0].copy_(self.off_obs[self.T])

    def iteration(self):
        """One PPO iteration; device time of rollout / update accumulates in self.timings (s)."""
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        self.rollout(defer_common=True)
        ev[1].record()
        losses = self.update()
        ev[2].record()
        self._pending_events.append(ev)
        self.iterations += 1
        if self.metric_bufs is not None:
            self._harvest_episodes()
        return losses

    # ---- metrics
    def _harvest_episodes(self):
        """Per-replica values of every episode finished by now (trainPPO.py:200-226), appended to
        self.episode_log; their accumulator slots are zeroed for reuse."""
        from . import metrics as mx
        s = self.env.shape
        done = self.rounds_done // self.ep_len
        while len(self.episode_log) < done:
            slot = len(self.episode_log) % self.metric_slots
            raw = torch.cat([b[slot] for b in self.metric_bufs]).cpu().numpy()
            for b in self.metric_bufs:
                b[slot].zero_()
            self.episode_log.append(mx.episode_values(mx.view(raw), self.cfg, self.ep_len, s.n_agents, s.n_cores,
                                                      s.collection_length))

    def args_dict(self, replica="mean", params=None):
        """argsDict of the finished episodes (trainPPO.py:229-243): replica = "mean" averages the
        replicas' values per episode, an int picks one replica."""
        from . import metrics as mx
        p = dict(params or {})
        p.setdefault("episodeLength", self.ep_len)
        p.setdefault("UPDATE_STEP", self.T)
        p.setdefault("n_envs", self.E * self.world_size)
        return mx.args_dict(self.episode_log, self.cfg, p, replica=replica)

    def save_args_dict(self, directory: str = ".", file_name: str = "data{}.pkl", replica="mean", params=None):
        """args_dict() pickled as the first free data{i}.pkl in directory (trainPPO.py:245-251)."""
        from . import metrics as mx
        return mx.save_args_dict(self.args_dict(replica, params), file_name, directory)

    @property
    def timings(self):
        for ev in self._pending_events:
            ev[2].synchronize()
            self._timings["rollout"] += ev[0].elapsed_time(ev[1]) / 1e3
            self._timings["update"] += ev[1].elapsed_time(ev[2]) / 1e3
        self._pending_events = []
        return self._timings

    @timings.setter
    def timings(self, value):
        self._pending_events = []
        self._timings = dict(value)

    def flags(self):
        return self.env.flags()
