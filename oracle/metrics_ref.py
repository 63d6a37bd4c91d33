"""The training driver's per-episode metrics, restated on the object-faithful world (pyref).

TEST INFRASTRUCTURE ONLY. Follows trainPPO.py:139-226 line for line (paths relative to
/root/reference/src), with the same container types: torch int64 accumulators of the unit rewards
(float64 once `+=` meets the float64 free-price arrays), a numpy int64 agent accumulator,
`statistics.mean` over the collected per-round values, and the world's `verweilzeiten` /
`acceptedOffers` lists. Checks marl-scheduling_amd/metrics.py + the env kernel's accumulators.
"""
from __future__ import annotations

import statistics
import warnings

import numpy as np
import torch


class EpisodeRecorder:
    """One env's episode as trainPPO.py collects it; feed every pyref step, then finish()."""

    def __init__(self, world, free_prices: bool):
        self.w = world
        self.free = free_prices
        N, C, L = world.N, world.C, world.L
        # trainPPO.py:145-157 (divided agents)
        self.core_acc = torch.tensor([[[0] for _ in range(L)] for _ in range(N)])
        self.price_acc = torch.tensor([[[0] for _ in range(L)] for _ in range(N)], dtype=float)
        self.acceptor_acc = torch.tensor([[[0] for _ in range(C)] for _ in range(N)])
        self.agent_acc = np.array([0 for _ in range(N)])
        self.prices, self.auct, self.qual, self.amount = [], [], [], []
        self.term_rev = 0
        self.dwell_start = len(world.dwell)

    def add(self, step_out):
        """step_out = pyref.PyWorld.step(...) return value."""
        _, rewards, qualities, _ = step_out
        offer_r, acc_r, auct_r, agent_r, term_rev = rewards
        for o in self.w.accepted:  # trainPPO.py:172-174
            self.prices.append((o.price, o.kind))
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            if self.free:  # trainPPO.py:176-180
                self.core_acc += offer_r[0]
                self.price_acc += offer_r[1]
            else:
                self.core_acc += offer_r
        self.agent_acc += agent_r
        self.acceptor_acc += acc_r
        self.auct.append(sum(auct_r.tolist()))
        # SchedulingEnvironment.py:189-192: (mean or None, count)
        if qualities:
            self.qual.append(statistics.mean(qualities))
        self.amount.append(len(qualities))
        self.term_rev += term_rev  # Reward.py:193

    def finish(self, cfg, episode_length: int):
        """The values trainPPO.py:200-226 appends at `done`."""
        w = self.w
        T, N, C = episode_length, w.N, w.C
        dw = w.dwell[self.dwell_start:]
        d = {}
        acc = []
        for i in range(len(cfg.priorities)):  # trainPPO.py:201-209
            v = [t[3] for t in dw if (t[0] == cfg.priorities[i]) & (t[1] == cfg.lengths[i])]
            acc.append(statistics.mean(v) if v != [] else None)
        d["dwellTimes"] = acc
        acc1 = []
        for i in range(len(cfg.priorities)):  # trainPPO.py:210-217
            lc = [tup[0] for tup in self.prices if tup[1] == i]
            acc1.append(statistics.mean(lc) if lc != [] else None)
        d["prices"] = acc1
        d["coreChooserRew"] = (self.core_acc / T).numpy().mean()
        d["priceChooserRew"] = (self.price_acc / T).numpy().mean()
        d["acceptorRew"] = (self.acceptor_acc / T).numpy().mean()
        d["auctioneerRew"] = statistics.mean(self.auct)
        d["acceptionQuality"] = statistics.mean(self.qual) if self.qual != [] else None
        d["acceptionAmount"] = statistics.mean(self.amount)
        d["agentRew"] = self.agent_acc / T
        d["tradeRevenues"] = 0 / (T * N * C)
        d["terminationRevenues"] = self.term_rev / (T * N * C)
        return d
