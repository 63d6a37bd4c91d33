"""Aggregated and fully-aggregated PPO agents over E env replicas (PPOAggregatedFixPriceEnv /
PPOFullyAggregatedFixPriceEnv, SchedulingEnvironment.py:213-250; Agent.py:73-140, 359-492).

An aggregated agent has one acceptor net over all its cores and one offer net over all its slots
(AggregatedAcceptorPPO / AggregatedOfferPPO, PPOmodules.py:177-210: 32 hidden units,
(O+1)^C and (C+1)^L actions); a fully aggregated agent has one net for both (FullyAggregatedPPO,
PPOmodules.py:213-232: 64 hidden units, (O+1)^C (C+1)^L actions). The world is the divided one,
so each round is

  aggregated obs (ms_aggregate_obs, HIP) -> act (ms_wide_act, HIP: the 32 / 64-hidden nets with
  (O+1)^C-sized softmaxes) -> decode the action numbers (ms_decode_aggregated, HIP) -> env step
  (ms_env_step, HIP, with the aggregated rewards of Reward.py:92-143 from the same settlement)

and UPDATE_STEP rounds are followed by PPO.update of every agent's nets (PPOmodules.py:127-174;
HIP returns kernel + the ms_wide_grad gradient + HIP Adam). Rewards saved per agent follow
SchedulingEnvironment.py:223-247: the acceptor net trains on agentReward, the offer net on the
aggregated offer reward, the fully aggregated net on their sum. The aggregated envs are
fixed-price only in the reference; so are these.
"""
from __future__ import annotations

import torch

from . import abi
from .env import BatchedEnv
from .ppo import PPOGroup, discounted_returns, reference_actor_critic_params
from .trainer import Hyper, env_seed

HIDDEN_AGGREGATED = 32  # AggregatedAcceptorPPO / AggregatedOfferPPO numberOfNeurons (PPOmodules.py:181,199)
HIDDEN_FULLY = 64       # FullyAggregatedPPO numberOfNeurons (PPOmodules.py:221)


class _AggUnit:
    """Rollout rings of one aggregated net type (one net per agent): obs [T+1][E][N][stride] int8,
    actions [T][E][N] int32, log-probs [T][E][N] f32, rewards [T][E][N] f32."""

    def __init__(self, name, T, E, N, dim, stride, group: PPOGroup, device):
        self.name, self.T, self.E, self.N, self.D, self.stride, self.group = name, T, E, N, dim, stride, group
        self.obs = torch.zeros((T + 1, E, N, stride), dtype=torch.int8, device=device)
        self.actions = torch.zeros((T, E, N), dtype=torch.int32, device=device)
        self.logprobs = torch.zeros((T, E, N), dtype=torch.float32, device=device)
        self.rewards = torch.zeros((T, E, N), dtype=torch.float32, device=device)

    def act(self, t):
        """Every agent's net on its E rows of round t (ms_wide_act), into the rings."""
        self.group.wide_act(self.obs[t], action=self.actions[t], logprob=self.logprobs[t])

    def batch(self):
        """The update's rows r = t*E + e: states [T*E, N, stride], actions / log-probs [T*E, N] (views of
        the rings) and the normalised returns [N, T*E]."""
        T, E, N = self.T, self.E, self.N
        ret = discounted_returns(self.rewards.reshape(T, E * N), self.group.gamma)  # [E*N, T]
        ret = ret.view(E, N, T).permute(1, 2, 0).reshape(N, T * E).contiguous()
        return (self.obs[:T].view(T * E, N, self.stride), self.actions.view(T * E, N),
                self.logprobs.view(T * E, N), ret)

    def update(self):
        losses = self.group.update_wide(*self.batch())
        self.group.sync_old()
        return torch.stack(losses)


class AggregatedTrainer:
    """The trainPPO.py loop (trainPPO.py:133-227) for aggregatedAgents / fullyAggregatedAgents."""

    def __init__(self, cfg: abi.MsConfig, n_envs: int, fully: bool = False, hyper: Hyper | None = None, seed: int = 0,
                 device=None):
        if cfg.free_prices:
            raise ValueError("the aggregated envs are fixed-price only (SchedulingEnvironment.py:213-248)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        torch.cuda.set_device(self.device)
        self.cfg, self.E, self.fully = cfg, int(n_envs), bool(fully)
        self.hp = hp = hyper or Hyper()
        T = self.T = hp.update_step
        self.env = BatchedEnv(cfg, self.E, seed=env_seed(seed, 0, self.E), device=self.device)
        env = self.env
        N, C, L = env.N, env.C, env.L
        self.N = N
        n_acc, n_off = env.aggregated_action_counts()
        if n_acc * n_off >= 2 ** 31:
            raise ValueError("aggregated action space (O+1)^C (C+1)^L = %d does not fit int32" % (n_acc * n_off))
        dims = env.aggregated_dims()
        max_len = max(cfg.job_length[: cfg.n_kinds])
        acc_gamma = hp.acceptor_gamma if hp.acceptor_gamma is not None else -((1 - max_len) / max_len) + 0.04
        K = max(hp.raw_k_epochs, 1)  # trainPPO.py:54-55,76-77: centralisation factor 1
        torch.manual_seed(seed)
        dev = self.device
        # nets in the reference's construction order: agent by agent, each PPO builds policy then
        # policy_old (PPOmodules.py:99,107); AggregatedFixPricePPOAgent: acceptor, then offer (Agent.py:363-366)
        if self.fully:
            A, D, H = n_acc * n_off, dims["fully"][0], HIDDEN_FULLY
            nets = []
            for _ in range(N):
                nets.append(reference_actor_critic_params(D, A, H))
                reference_actor_critic_params(D, A, H)
            grp = PPOGroup(N, D, A, hp.lr_actor, hp.lr_critic, acc_gamma, hp.eps_clip, K, dev, init_nets=nets, hidden=H)
            self.units = {"fully": _AggUnit("fully", T, self.E, N, D, dims["fully"][1], grp, dev)}
        else:
            H = HIDDEN_AGGREGATED
            da, do = dims["acceptor"][0], dims["offer"][0]
            acc_nets, off_nets = [], []
            for _ in range(N):
                acc_nets.append(reference_actor_critic_params(da, n_acc, H))
                reference_actor_critic_params(da, n_acc, H)
                off_nets.append(reference_actor_critic_params(do, n_off, H))
                reference_actor_critic_params(do, n_off, H)
            ga = PPOGroup(N, da, n_acc, hp.lr_actor, hp.lr_critic, acc_gamma, hp.eps_clip, K, dev, init_nets=acc_nets,
                          hidden=H)
            go = PPOGroup(N, do, n_off, hp.lr_actor, hp.lr_critic, hp.offer_gamma, hp.eps_clip, K, dev,
                          init_nets=off_nets, hidden=H)
            self.units = {"acceptor": _AggUnit("acceptor", T, self.E, N, da, dims["acceptor"][1], ga, dev),
                          "offer": _AggUnit("offer", T, self.E, N, do, dims["offer"][1], go, dev)}
        self.div_obs = env.obs_buffers()
        self.rew = env.reward_buffers(aggregated=True)
        self.numbers = torch.zeros(((1 if self.fully else 2), self.E, N), dtype=torch.int32, device=dev)
        self.n_bad = torch.zeros(1, dtype=torch.int32, device=dev)
        env.reset(self.div_obs)
        self._aggregate(0)
        self.iterations = 0

    def _aggregate(self, t):
        out = {k: u.obs[t] for k, u in self.units.items()}
        self.env.aggregate_obs(self.div_obs, out=out)

    def round(self, t: int):
        """getActionForAllAgents + auctioneer + env.step + saveRewards (trainPPO.py:160-167)."""
        for u in self.units.values():
            u.act(t)
        if self.fully:
            self.numbers[0].copy_(self.units["fully"].actions[t])
        else:
            self.numbers[0].copy_(self.units["acceptor"].actions[t])
            self.numbers[1].copy_(self.units["offer"].actions[t])
        # n_bad counts illegal action numbers over the iteration (reset at its start); the reference
        # raises on one (Agent.py:651-652): iteration() checks the count after the rollout
        acc, off = self.env.decode_aggregated(self.numbers, self.fully, n_bad=self.n_bad)
        self.env.step(acc, off, obs=self.div_obs, rewards=self.rew)
        agent = self.rew["agent"].float()
        agg_off = self.rew["aggregated_offer"].float()
        if self.fully:  # PPOFullyAggregatedFixPriceEnv.saveRewards (SchedulingEnvironment.py:243-247)
            self.units["fully"].rewards[t].copy_(agent + agg_off)
        else:  # PPOAggregatedFixPriceEnv.saveRewards (SchedulingEnvironment.py:223-225, Agent.py:388-390)
            self.units["acceptor"].rewards[t].copy_(agent)
            self.units["offer"].rewards[t].copy_(agg_off)
        self._aggregate(t + 1)

    def update(self):
        """env.updateAgents(): every agent's nets (Agent.py:384-386, 487-488)."""
        losses = {k: u.update() for k, u in self.units.items()}
        for u in self.units.values():
            u.obs[0].copy_(u.obs[self.T])
        return losses

    def iteration(self):
        self.n_bad.zero_()
        for t in range(self.T):
            self.round(t)
        if int(self.n_bad.item()):
            raise ValueError("Illegal Argument: %d action numbers outside the action space (Agent.py:651-652)"
                             % int(self.n_bad.item()))
        self.iterations += 1
        return self.update()

    def flags(self) -> int:
        return self.env.flags()

    def bad_actions(self) -> int:
        return int(self.n_bad.item())
