"""Drop-in ``SchedulingEnvironment`` module: the reference's PPO env classes on the HIP device.

The class names, constructor signatures and methods are those of
SchedulingEnvironment.py:21-348:

* ``reset()`` and ``step(offerActions, acceptorActions, auctioneer_action)``
  return the same tuples. Observations are nested lists of 1-D ``torch.int64``
  CPU tensors. Rewards are numpy arrays shaped ``[N][L][1]`` / ``[N][C][1]`` /
  ``[C]`` / ``[N]``; the free-price offer rewards are a ``(coreChooser,
  priceChooser)`` pair of float64 arrays. The 8th element is
  ``(acceptionQualityMean | None, count)`` and the 9th is ``done``.
* ``getActionForAllAgents(accObs, offObs)`` returns
  ``(acceptorActions[N][C], offerActions[N][L])``; free-price offer actions are
  ``(coreChooserAction, price)`` tuples.
* ``saveRewards(...)`` and ``updateAgents()`` follow the reference.

Every round runs on libmarlsched at E = 1 (see ``marlsched_dropin``). The
aggregated, fully-aggregated, hard-coded-agent and DQN envs are outside this
build's hot path and raise ``NotImplementedError``.

``LocallySharedParamsDividedFreePriceEnv`` is an addition. BASELINE cfg3 trains
free prices with locally shared parameters, which the reference has no class
for. It combines ``LocallySharedPPO`` (PPOmodules.py:490-597) with
``FreePriceOfferPPO`` (:273-332) and the free-price rewards (Reward.py:6-89).
"""
from __future__ import annotations

import random

import numpy as np
import torch

from marlsched_dropin import Engine, Units, acception_quality, ppo, reference_nets

__all__ = [
    "SchedulingEnv", "PPOSchedulingEnv", "PPODividedFixedPriceEnv", "PPODividedFreePriceEnv",
    "GloballySharedParamsDividedFixedPriceEnv", "LocallySharedParamsDividedFixedPriceEnv",
    "LocallySharedParamsDividedFreePriceEnv", "PPOAggregatedFixPriceEnv", "PPOFullyAggregatedFixPriceEnv",
    "HardcodedFixPriceEnvironment", "DQNDividedFixedPricesEnv",
]


class _AgentHandle:
    """world.agents entries: the reference's Agent objects keep their nets; here the nets of all
    agents are grouped per unit type in the env, so an agent only carries its ID."""

    def __init__(self, agent_id):
        self.agentID = agent_id


class SchedulingEnv:
    """SchedulingEnv (SchedulingEnvironment.py:21-192)."""

    _free = False
    _commercial = True

    def __init__(self, world, params):
        self.world = world
        self.formerCorePrios = [-1 for _ in range(world.numberOfCores)]
        self.formerCoreLengths = [-1 for _ in range(world.numberOfCores)]
        self.netZeroOfferReward = params["netZeroOfferReward"]
        self.tradeRevenues = 0
        self.terminationRevenues = 0
        self._eng = Engine(world, self._free, self._commercial, self.netZeroOfferReward)
        world._attach(self._eng)
        world.agents = [_AgentHandle(i + 1) for i in range(world.numberOfAgents)]

    def reset(self):
        return self._eng.reset()

    def step(self, offerActions, acceptorActions, auctioneer_action):
        eng, w = self._eng, self.world
        (acc_obs, off_obs, auct_obs), offers, terms, r, round_before = eng.step(offerActions, acceptorActions,
                                                                                auctioneer_action)
        w._record(offers, terms, round_before)
        quality = acception_quality(w.acceptedOffers, self.formerCorePrios, self.formerCoreLengths)
        offerRewards, acceptorRewards, auctioneerReward, agentReward = self._rewards(r, terms)
        done = (w.round % w.episodeLength) == 0
        # formerCorePrios/Lengths = the cores' (prio, rem) after this round: the first 2C values of any
        # offer observation row (Agent.py:271-300; an empty core reads -1, -1)
        row = off_obs[0][0]
        C = w.numberOfCores
        self.formerCorePrios = [int(row[2 * c]) for c in range(C)]
        self.formerCoreLengths = [int(row[2 * c + 1]) for c in range(C)]
        return (acc_obs, off_obs, auct_obs, offerRewards, acceptorRewards, auctioneerReward, agentReward, quality,
                done)

    def _rewards(self, r, terms):
        """getDividedFixedPricesReward (Reward.py:146-212) containers."""
        N, C, L = self.world.numberOfAgents, self.world.numberOfCores, self.world.collectionLength
        off = np.rint(r["offer"]).astype(np.int64).reshape(N, L, 1)
        acc = r["acceptor"].astype(np.int64).reshape(N, C, 1)
        auct = r["auctioneer"].astype(np.int64).reshape(C)
        agent = r["agent"].astype(np.int64).reshape(N)
        self.terminationRevenues += sum(self.world.rewardMultiplier * t[2] for t in terms)
        return off, acc, auct, agent

    def render(self, mode="human"):
        print("___________________________________")
        print("Round: ")
        print(self.world.round)
        if mode == "human":
            print("Core-States:")
            for core in self.world.cores:
                print(core.getCoreState())
        print("Offer-States:")
        for offer in self.world.offers:
            print(offer.getOfferState())
        print("Accepted Offers:")
        for offer in self.world.acceptedOffers:
            print("coreID: {}, offererID: {}, recipientID: {}, offeredReward {}, slot: {}".format(
                offer.coreID, offer.offererID, offer.recipientID, offer.offeredReward, offer.queuePosition))

    def close(self):
        pass

    def plotResult(self, argsDict):
        raise NotImplementedError("plotting (Plot.py) is outside this build's hot path")


class PPOSchedulingEnv(SchedulingEnv):
    """PPOSchedulingEnv (SchedulingEnvironment.py:195-210) + the unit nets of all agents, grouped.

    arch: "divided" (one net per unit), "local" (one net per agent and unit type),
    "global" (one net per unit type)."""

    _arch = "divided"

    def __init__(self, world, params):
        super().__init__(world, params)
        self.LR_ACTOR = params["LR_ACTOR"]
        self.LR_CRITIC = params["LR_CRITIC"]
        self.OFFER_GAMMA = params["OFFER_GAMMA"]
        self.ACCEPTOR_GAMMA = params["ACCEPTOR_GAMMA"]
        self.EPS_CLIP = params["EPS_CLIP"]
        self.RAW_K_EPOCHS = params["RAW_K_EPOCHS"]
        self.ACCEPTOR_K_EPOCHS = params["ACCEPTOR_K_EPOCHS"]
        self.OFFER_K_EPOCHS = params["OFFER_K_EPOCHS"]
        self.CENTRALISATION_SAMPLE = params["CENTRALISATION_SAMPLE"]
        self._build_nets()
        self._seed = torch.initial_seed() & ((1 << 63) - 1)
        self._ctr = 0

    # ---- nets in the reference's construction order
    def _build_nets(self):
        w, eng = self.world, self._eng
        N, C, L = w.numberOfAgents, w.numberOfCores, w.collectionLength
        s = eng.env.shape
        dims = dict(acc=(s.acc_obs_dim, s.acc_actions), off=(s.off_obs_dim, s.off_actions),
                    price=(4, s.price_actions))
        off_units = ["off", "price"] if self._free else ["off"]
        if self._arch == "divided":  # Agent.py:495-502, 589-596 (FreePriceOfferPPO: coreChooser, priceChooser)
            order = [u for _ in range(N) for u in ["acc"] * C + off_units * L]
            groups = dict(acc=N * C, off=N * L, price=N * L)
        elif self._arch == "local":  # Agent.py:669-680: LocallySharedAcceptorPPO, then the offer net
            order = [u for _ in range(N) for u in ["acc"] + off_units]
            groups = dict(acc=N, off=N, price=N)
        else:  # SchedulingEnvironment.py:269-275: sharedAcceptorNet, sharedOfferNet
            order = ["acc"] + off_units
            groups = dict(acc=1, off=1, price=1)
        nets = reference_nets(order, {k: dims[k] for k in set(order)})
        if self._free:
            k_off = self.RAW_K_EPOCHS if self._arch == "divided" else self.OFFER_K_EPOCHS
        else:
            k_off = self.OFFER_K_EPOCHS
        gam = dict(acc=self.ACCEPTOR_GAMMA, off=self.OFFER_GAMMA, price=self.OFFER_GAMMA)
        kk = dict(acc=self.ACCEPTOR_K_EPOCHS, off=k_off, price=k_off)
        n_units = dict(acc=N * C, off=N * L, price=N * L)
        strides = dict(acc=s.acc_obs_stride, off=s.off_obs_stride, price=4)
        self._units = {}
        for k in ["acc"] + off_units:
            D, A = dims[k]
            grp = ppo.PPOGroup(groups[k], D, A, self.LR_ACTOR, self.LR_CRITIC, gam[k], self.EPS_CLIP, kk[k],
                               eng.device, init_nets=nets[k])
            self._units[k] = Units(grp, n_units[k], strides[k], eng.device)
        self._env_price = torch.zeros((1, N * L), dtype=torch.int8, device=eng.device)

    # ---- getActionForAllAgents (SchedulingEnvironment.py:150-172 + Agent.getActions)
    def _device_rows(self, nested, stride, d):
        """Observation rows on the device: the env's own buffer when the driver passes back the
        observation it got from reset/step, else the given tensors."""
        rows = torch.stack([torch.as_tensor(x) for agent in nested for x in agent]).to(torch.int8)
        out = torch.zeros((rows.shape[0], stride), dtype=torch.int8)
        out[:, :d] = rows
        return out.to(self._eng.device)

    def getActionForAllAgents(self, nestedAcceptorNetObservationTensors, nestedOfferNetObservationTensors):
        eng, w = self._eng, self.world
        N, C, L = w.numberOfAgents, w.numberOfCores, w.collectionLength
        last = eng.last_obs
        if last is not None and nestedAcceptorNetObservationTensors is last[0]:
            acc_rows = eng.obs["acceptor"][0].view(N * C, -1)
        else:
            acc_rows = self._device_rows(nestedAcceptorNetObservationTensors, eng.obs["acceptor"].shape[-1], eng.d_acc)
        if last is not None and nestedOfferNetObservationTensors is last[1]:
            off_rows = eng.obs["offer"][0].view(N * L, -1)
        else:
            off_rows = self._device_rows(nestedOfferNetObservationTensors, eng.obs["offer"].shape[-1], eng.d_off)
        base = self._ctr
        self._ctr += 8
        ua, uo = self._units["acc"], self._units["off"]
        ta, to = ua.next_slot(), uo.next_slot()
        ua.states[ta].copy_(acc_rows)
        uo.states[to].copy_(off_rows)
        if self._free:
            up = self._units["price"]
            tp = up.next_slot()
            out = dict(core_action=uo.actions[to].view(1, -1), core_logprob=uo.logprobs[to].view(1, -1),
                       price_state=up.states[tp].view(1, N * L, 4), price_action=up.actions[tp].view(1, -1),
                       price_logprob=up.logprobs[tp].view(1, -1), env_price=self._env_price)
            ppo.offer_act_free(uo.group.policy_old, up.group.policy_old, uo.states[to].unsqueeze(0), C, self._seed,
                               base + 1, out)
            up.T += 1
        else:
            uo.group.policy_old.act(uo.states[to].unsqueeze(0), N * L, self._seed, base + 1,
                                    action=uo.actions[to].view(1, -1), logprob=uo.logprobs[to].view(1, -1))
        ua.group.policy_old.act(ua.states[ta].unsqueeze(0), N * C, self._seed, base + 3,
                                action=ua.actions[ta].view(1, -1), logprob=ua.logprobs[ta].view(1, -1))
        ua.T += 1
        uo.T += 1
        acc_a = ua.actions[ta].cpu().tolist()
        off_a = uo.actions[to].cpu().tolist()
        acc_l = [[int(acc_a[a * C + c]) for c in range(C)] for a in range(N)]
        if self._free:
            price = self._env_price[0].cpu().tolist()
            off_l = [[(int(off_a[a * L + j]), int(price[a * L + j])) for j in range(L)] for a in range(N)]
        else:
            off_l = [[int(off_a[a * L + j]) for j in range(L)] for a in range(N)]
        return acc_l, off_l

    # ---- saveRewards (SchedulingEnvironment.py:264-342; Agent.py:531-536, 610-619, 701-706)
    def saveRewards(self, offerNetRewards, acceptorNetRewards, agentReward):
        if self._free:
            self._units["off"].rewards.append(np.asarray(offerNetRewards[0], dtype=np.float64).reshape(-1))
            self._units["price"].rewards.append(np.asarray(offerNetRewards[1], dtype=np.float64).reshape(-1))
        else:
            self._units["off"].rewards.append(np.asarray(offerNetRewards, dtype=np.float64).reshape(-1))
        self._units["acc"].rewards.append(np.asarray(acceptorNetRewards, dtype=np.float64).reshape(-1))

    # ---- updateAgents (SchedulingEnvironment.py:208-210, 314-329; Agent.py:524-529, 603-608, 708-728)
    def updateAgents(self):
        w = self.world
        N, C, L, CS = w.numberOfAgents, w.numberOfCores, w.collectionLength, self.CENTRALISATION_SAMPLE
        off_types = ["off", "price"] if self._free else ["off"]
        if self._arch == "divided":
            sel = dict(acc=[list(range(N * C))], off=[list(range(N * L))])
        elif self._arch == "local":
            acc_d, off_d = [], []
            for _ in range(N):  # agent by agent: acceptor draws, then offer draws
                acc_d.append([random.randint(0, C - 1) for _ in range(CS)])
                off_d.append([random.randint(0, L - 1) for _ in range(CS)])
            sel = dict(acc=[[a * C + acc_d[a][i] for a in range(N)] for i in range(CS)],
                       off=[[a * L + off_d[a][i] for a in range(N)] for i in range(CS)])
        else:
            acc_s, off_s = [], []
            for _ in range(CS):
                a = random.randint(0, N - 1)
                acc_s.append([a * C + random.randint(0, C - 1)])
            for _ in range(CS):
                a = random.randint(0, N - 1)
                off_s.append([a * L + random.randint(0, L - 1)])
            sel = dict(acc=acc_s, off=off_s)
        losses = {}
        for k in ["acc"] + off_types:
            u = self._units[k]
            ls = []
            for s in sel["acc" if k == "acc" else "off"]:
                ls += u.update(s)
            u.clear()
            u.group.sync_old()
            losses[k] = ls
        self._last_losses = losses


class PPODividedFixedPriceEnv(PPOSchedulingEnv):
    """PPODividedFixedPriceEnv (SchedulingEnvironment.py:249-264)."""

    _arch = "divided"


class PPODividedFreePriceEnv(PPOSchedulingEnv):
    """PPODividedFreePriceEnv (SchedulingEnvironment.py:232-246)."""

    _arch = "divided"
    _free = True

    def __init__(self, world, params, commercialFreePriceReward):
        self._commercial = bool(commercialFreePriceReward)
        self.commercialFreePriceReward = commercialFreePriceReward
        super().__init__(world, params)

    def _rewards(self, r, terms):
        """getDividedFreePricesReward (Reward.py:6-89) containers."""
        N, C, L = self.world.numberOfAgents, self.world.numberOfCores, self.world.collectionLength
        core = r["offer"].astype(np.float64).reshape(N, L, 1)
        price = r["price"].astype(np.float64).reshape(N, L, 1)
        acc = r["acceptor"].astype(np.int64).reshape(N, C, 1)
        auct = r["auctioneer"].astype(np.int64).reshape(C)
        agent = r["agent"].astype(np.int64).reshape(N)
        return (core, price), acc, auct, agent


class GloballySharedParamsDividedFixedPriceEnv(PPOSchedulingEnv):
    """GloballySharedParamsDividedFixedPriceEnv (SchedulingEnvironment.py:267-306)."""

    _arch = "global"


class LocallySharedParamsDividedFixedPriceEnv(PPOSchedulingEnv):
    """LocallySharedParamsDividedFixedPriceEnv (SchedulingEnvironment.py:332-348)."""

    _arch = "local"


class LocallySharedParamsDividedFreePriceEnv(PPODividedFreePriceEnv):
    """Free prices with locally shared nets (BASELINE cfg3; not a reference class, see module doc)."""

    _arch = "local"


def _out_of_scope(name):
    class _Env:
        def __init__(self, *a, **k):
            raise NotImplementedError("%s is outside this build's hot path (DESIGN.md §8)" % name)

    _Env.__name__ = name
    return _Env


PPOAggregatedFixPriceEnv = _out_of_scope("PPOAggregatedFixPriceEnv")
PPOFullyAggregatedFixPriceEnv = _out_of_scope("PPOFullyAggregatedFixPriceEnv")
HardcodedFixPriceEnvironment = _out_of_scope("HardcodedFixPriceEnvironment")
DQNDividedFixedPricesEnv = _out_of_scope("DQNDividedFixedPricesEnv")
