"""Drop-in ``world`` module: ``World(params)`` with the reference's attributes (world.py:210-254).

The state itself lives on the HIP device once an env class from
``SchedulingEnvironment`` is constructed on this world. ``World`` keeps the
constructor parameters, the per-round records the driver reads
(``round``, ``acceptedOffers``, ``verweilzeiten``, ``jobTerminationInfo``) and
read-only views of cores and offers for ``render``.
"""
from __future__ import annotations

import random  # noqa: F401  (the reference driver relies on `from world import *` bringing it in)
from collections import deque  # noqa: F401
from fractions import Fraction as F  # noqa: F401  (trainPPO.py:53 uses F via `from world import *`)

from marlsched_dropin import AcceptedOffer, CoreView, JobView, Verweilzeit

__all__ = ["World", "Verweilzeit", "F", "random", "deque"]


class _AuctioneerHandle:
    """world.auctioneer: Auctioneer.getAuctioneerAction (Auctioneer.py:95-102) on the device."""

    auctioneerID = 0

    def __init__(self, world):
        self.world = world

    def getAuctioneerAction(self, auctioneerObservationsTensor):
        # The hard-coded auctioneer reads the env's current state, which is what the observation
        # returned by the last reset/step describes; its tie-breaks draw from `random`.
        return self.world._engine().auctioneer_actions()


class World(object):
    def __init__(self, params):
        self.freePrices = params["freePrices"]
        if self.freePrices is False:
            self.listOfFixPrices = params["fixPricesList"]
        self.numberOfAgents = params["numberOfAgents"]
        self.numberOfCores = params["numberOfCores"]
        self.possibleJobLengths = params["possibleJobLengths"]
        self.possibleJobPriorities = params["possibleJobPriorities"]
        self.probabilities = params["probabilities"]
        self.accProbabilities = [sum(self.probabilities[: (i + 1)]) for i in range(len(self.probabilities))]
        self.maxSumToOffer = max(self.possibleJobPriorities)
        self.collectionLength = params["collectionLength"]
        self.maxAmountOfOffers = self.numberOfAgents * self.collectionLength
        self.maxAmountOfOffersToOneAgent = self.numberOfAgents * self.collectionLength
        self.maxAmountOfAcceptionsPerTimeStepPerAgent = min(self.maxAmountOfOffersToOneAgent, self.numberOfCores)
        self.newJobsPerRoundPerAgent = params["newJobsPerRoundPerAgent"]
        self.episodeLength = params["episodeLength"]
        self.maxVisibleOffers = params["maxVisibleOffers"]
        self.rewardMultiplier = params["rewardMultiplier"]
        self.jobTerminationInfo = []
        self.verweilzeiten = []
        self.acceptedOffers = []
        self.agents = None
        self.randomPolicy = False
        self.auctioneer = _AuctioneerHandle(self)
        self._eng = None

    # ---- device engine (attached by the env constructor)
    def _attach(self, engine):
        self._eng = engine

    def _engine(self):
        if self._eng is None:
            raise RuntimeError("construct an env from SchedulingEnvironment on this World first")
        return self._eng

    @property
    def round(self) -> int:
        return self._eng.round if self._eng is not None else 0

    def _record(self, offers, terminations, round_before):
        """The per-round lists World.step1 rebuilds (world.py:309-313, 285-293, 336-357)."""
        self.acceptedOffers = offers
        self.jobTerminationInfo = []
        mult = self.rewardMultiplier
        for core_id, owner, prio, init_len, dwell in terminations:
            core = CoreView(core_id, owner, JobView(prio, 0, init_len))
            self.jobTerminationInfo.append((core, owner, None, mult * prio, round_before + 1))
            self.verweilzeiten.append(Verweilzeit(prio, init_len, dwell, (dwell - 1) / init_len))

    # ---- read-only views of the device state (render / inspection)
    @property
    def cores(self):
        s = self._engine().export()
        prio = self.possibleJobPriorities
        out = []
        for c in range(self.numberOfCores):
            k = int(s["core_kind"][0, c])
            job = JobView() if k < 0 else JobView(prio[k], int(s["core_rem"][0, c]), self.possibleJobLengths[k], k,
                                                  int(s["core_birth"][0, c]), int(s["core_owner"][0, c]))
            out.append(CoreView(c + 1, int(s["core_owner"][0, c]), job))
        return out

    @property
    def offers(self):
        s = self._engine().export()
        out = []
        N, L = self.numberOfAgents, self.collectionLength
        for a in range(N):
            for j in range(L):
                c = int(s["offer_core"][0, a, j])
                if c >= 0:
                    k = int(s["slot_kind"][0, a, j])
                    out.append(AcceptedOffer(a + 1, int(s["offer_recip"][0, a, j]), c + 1, j,
                                             int(s["offer_price"][0, a, j]), int(s["slot_rem"][0, a, j]),
                                             self.possibleJobPriorities[k], k, self.round - 1))
        return out
