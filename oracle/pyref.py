"""Object-faithful pure-Python restatement of the marl-scheduling step.

TEST INFRASTRUCTURE ONLY — used by tests/ to cross-check the C restatement
(oracle/ms_oracle.c) on small cases. It keeps the reference's object graph and
iteration orders (paths relative to /root/reference/src): jobs and cores as
objects, a flat offer list in creation order, per-core liability deques with
appendleft, the global-stream random draws (here a ``random.Random`` instance
seeded like ``random.seed``), and numpy int64/float64 reward arrays shaped like
Reward.py. Parity status: unpinned against reference outputs (the reference has
no fixtures and executing it was denied); see DESIGN.md.
"""
from __future__ import annotations

import random
from collections import deque
from dataclasses import dataclass, field

import numpy as np


@dataclass
class Job:  # world.py:79-104
    empty: bool = True
    owner: int = -1
    prio: int = -1
    rem: int = -1
    init_len: int = -1
    birth: int = -1
    kind: int = -1
    wait: bool = False


@dataclass
class Offer:  # world.py:156-196
    offer_id: int
    offerer: int
    recipient: int
    core_id: int
    queue_pos: int
    price: int
    nec_time: int
    prio1: int
    kind: int
    round: int


@dataclass
class Config:
    n_agents: int
    n_cores: int
    collection_length: int
    priorities: list
    lengths: list
    probabilities: list
    fix_prices: list = field(default_factory=list)
    free_prices: bool = False
    commercial: bool = True
    net_zero_offer_reward: float = 0.5
    new_jobs: int = 1
    reward_multiplier: int = 1
    episode_length: int = 100


def ratio(p, n):  # HardcodedModules.py:5-13
    if p == -1 or n == -1 or p == -2 or n == -2:
        return -1
    return p / n


class PyWorld:
    """World + divided env façade (world.py:210-478, SchedulingEnvironment.py:32-192)."""

    def __init__(self, cfg: Config, seed: int):
        self.cfg = cfg
        self.N, self.C, self.L = cfg.n_agents, cfg.n_cores, cfg.collection_length
        self.O = self.N * self.L
        self.acc = [sum(cfg.probabilities[: i + 1]) for i in range(len(cfg.probabilities))]
        self.core_job = [Job() for _ in range(self.C)]
        self.core_owner = [0] * self.C
        self.coll = [[Job() for _ in range(self.L)] for _ in range(self.N)]
        self.free = [self.L] * self.N
        self.offers: list[Offer] = []
        self.liab = [deque() for _ in range(self.C)]
        self.round = 0
        self.former_prio = [-1] * self.C
        self.former_len = [-1] * self.C
        self.rng = random.Random(seed)
        self.accepted: list[Offer] = []
        self.term = []
        self.dwell = []
        self.spawn_edge = 0

    @classmethod
    def from_state(cls, cfg: Config, st: dict, mt_words, mt_index):
        """A world in a given state (the KAT fixture's form, tests/golden/make_kats.py): cores, slots,
        the pending offer of each slot (IDs in slot order, made last round), the liability deques
        newest first, the CPython random state. formerCorePrios/Lengths are the cores' jobs as the
        previous step left them (SchedulingEnvironment.py:64-66), i.e. this state's."""
        w = cls(cfg, 0)
        N, C, L = w.N, w.C, w.L
        rnd = int(st["round"])
        w.round = rnd
        for c in range(C):
            k = int(st["core_kind"][c])
            if k >= 0:
                w.core_job[c] = Job(False, int(st["core_owner"][c]), cfg.priorities[k], int(st["core_rem"][c]),
                                    cfg.lengths[k], int(st["core_birth"][c]), k)
            w.core_owner[c] = int(st["core_owner"][c])
        w.former_prio = [j.prio for j in w.core_job]
        w.former_len = [j.rem for j in w.core_job]
        for a in range(N):
            for q in range(L):
                k = int(st["slot_kind"][a][q])
                if k >= 0:
                    w.coll[a][q] = Job(False, a + 1, cfg.priorities[k], int(st["slot_rem"][a][q]), cfg.lengths[k],
                                       int(st["slot_birth"][a][q]), k, bool(st["slot_wait"][a][q]))
            w.free[a] = sum(1 for j in w.coll[a] if j.empty)
        oid = 1
        for a in range(N):
            for q in range(L):
                c = int(st["offer_core"][a][q])
                if c >= 0:
                    j = w.coll[a][q]
                    w.offers.append(Offer(oid, a + 1, int(st["offer_recip"][a][q]), c + 1, q,
                                          int(st["offer_price"][a][q]), j.rem, j.prio, j.kind, rnd - 1))
                    oid += 1
        for c, chain in enumerate(st["liab"]):
            w.liab[c] = deque(Offer(0, int(e[0]), int(e[1]), c + 1, 0, int(e[2]), int(e[3]), 0, -1, int(e[4]))
                              for e in chain)
        w.rng.setstate((3, tuple(int(x) for x in mt_words) + (int(mt_index),), None))
        return w

    # ---- collections (world.py:123-141)
    def _insert(self, a, job):
        if self.free[a] <= 0:
            raise RuntimeError("collection full")
        for s in range(self.L):
            if self.coll[a][s].empty:
                self.coll[a][s] = job
                self.free[a] -= 1
                return

    def _remove(self, a, s):
        job = self.coll[a][s]
        self.coll[a][s] = Job()
        self.free[a] += 1
        return job

    # ---- offers addressed to (recipient, core) in ID order (Agent.py:178-197)
    def _offers_to(self, recipient, core_id):
        return [o for o in self.offers if o.recipient == recipient and o.core_id == core_id]

    def ids(self, recipient, core_id):
        ids = [o.offer_id for o in self._offers_to(recipient, core_id)]
        return ids + [-2] * (self.O - len(ids))

    # ---- world.executeAnOffer (world.py:261-293)
    def _execute(self, offer_id):
        off = next(o for o in self.offers if o.offer_id == offer_id)
        c = off.core_id - 1
        if off.recipient != self.core_owner[c]:
            return
        job = self._remove(off.offerer - 1, off.queue_pos)
        job.wait = False
        old = self.core_job[c]
        old = Job() if old.empty else old
        self.core_job[c] = job
        self.core_owner[c] = 0 if job.empty else job.owner
        if off.recipient != 0:
            self._insert(off.recipient - 1, old)
        entry = Offer(**vars(off))
        entry.round = self.round
        self.liab[c].appendleft(entry)
        self.accepted.append(Offer(**vars(off)))

    # ---- HardcodedAuctioneerAcceptor (HardcodedModules.py:54-78)
    def auctioneer_actions(self):
        out = []
        for c in range(self.C):
            obs = self.auctioneer_obs(c)
            if obs[0] == 0:
                out.append(self.O)
                continue
            own = ratio(obs[1], obs[2])
            pairs = list(zip(obs[3::2], obs[4::2]))
            rs = [ratio(p, n) for p, n in pairs]
            if max(rs) > own:
                cands = [(i, r) for i, r in enumerate(rs) if r == max(rs)]
                out.append(self.rng.sample(cands, 1)[0][0])
            else:
                out.append(self.O)
        return out

    # ---- DividedHardcodedAgent.getActions (Agent.py:630-641) of every agent on the env stream:
    #      per agent its HardcodedOfferers (HardcodedModules.py:81-109), then its HardcodedAcceptors (:16-45)
    def hardcoded_agent_actions(self):
        acc_obs = [[self.acceptor_obs(a, c) for c in range(self.C)] for a in range(self.N)]
        off_obs = [[self.offer_obs(a, s) for s in range(self.L)] for a in range(self.N)]
        acc_act, off_act = [], []
        for a in range(self.N):
            offers = []
            for s in range(self.L):
                row = off_obs[a][s]
                core_ratios = [ratio(row[2 * c], row[2 * c + 1]) for c in range(self.C)]
                low = min(core_ratios)
                cands = [(i, r) for i, r in enumerate(core_ratios) if r == low]
                offers.append(self.rng.sample(cands, 1)[0][0])
            accs = []
            for c in range(self.C):
                row = acc_obs[a][c]
                if row[0] == 0:
                    accs.append(self.O)
                    continue
                own = ratio(row[1], row[2])
                offered = [ratio(row[3 + 2 * k], row[4 + 2 * k]) for k in range(self.O)]
                best = max(offered)
                if best > own:
                    cands = [(i, r) for i, r in enumerate(offered) if r == best]
                    accs.append(self.rng.sample(cands, 1)[0][0])
                else:
                    accs.append(self.O)
            off_act.append(offers)
            acc_act.append(accs)
        return acc_act, off_act

    # ---- world.step1 (world.py:295-334) + SchedulingEnv.step (SchedulingEnvironment.py:32-83)
    def step(self, acc_act, off_act, auct_act=None):
        if auct_act is None:
            auct_act = self.auctioneer_actions()
        ids_now = [[self.ids(a + 1, c + 1) for c in range(self.C)] for a in range(self.N)]
        auct_ids = [self.ids(0, c + 1) for c in range(self.C)]
        for _ in self.term:
            pass  # liability resets already done in the last getRewards
        self.term = []
        self.accepted = []
        for a in range(self.N):
            for c in range(self.C):
                idx = int(acc_act[a][c])
                if idx < self.O:
                    oid = ids_now[a][c][idx]
                    if oid > 0:
                        self._execute(oid)
                else:
                    assert idx == self.O
        for c in range(self.C):
            idx = int(auct_act[c])
            if idx < self.O:
                oid = auct_ids[c][idx]
                if oid > 0:
                    self._execute(oid)
            else:
                assert idx == self.O
        # processOneTimestepAndUpdateOwnership (world.py:336-367)
        for c in range(self.C):
            job = self.core_job[c]
            if not job.empty:
                job.rem -= 1
                if job.rem == 0:
                    reward = self.cfg.reward_multiplier * job.prio
                    self.term.append((c, self.core_owner[c], reward, self.round + 1))
                    self.dwell.append(
                        (job.prio, job.init_len, self.round - job.birth,
                         (self.round - job.birth - 1) / job.init_len))
                    self.core_job[c] = Job()
                    self.core_owner[c] = 0
        # offers (world.py:406-478)
        self.offers = []
        next_id = 1
        for a in range(self.N):
            for s in range(self.L):
                act = off_act[a][s]
                if self.cfg.free_prices:
                    core_id, price = act[0] + 1, act[1]
                else:
                    core_id = act + 1
                    price = self.cfg.fix_prices[self.coll[a][s].kind]
                job = self.coll[a][s]
                if 1 <= core_id <= self.C and not job.empty and not job.wait:
                    self.offers.append(Offer(next_id, a + 1, self.core_owner[core_id - 1], core_id, s,
                                             price, job.rem, job.prio, job.kind, self.round))
                    next_id += 1
                    job.wait = True
                else:
                    job.wait = False
        # fillQueuesWithNewRandomJobs (world.py:369-376, Agent.py:50-70)
        k = self.cfg.new_jobs
        for a in range(self.N):
            owned = sum(1 for c in range(self.C) if self.core_owner[c] == a + 1)
            if owned + k <= self.free[a]:
                for _ in range(k):
                    u = self.rng.random()
                    kind = None
                    for i, p in enumerate(self.acc):
                        if u < p:
                            kind = i
                            break
                    if kind is None:
                        kind = len(self.acc) - 1
                        self.spawn_edge += 1
                    self._insert(a, Job(False, a + 1, self.cfg.priorities[kind], self.cfg.lengths[kind],
                                        self.cfg.lengths[kind], self.round, kind))
        self.round += 1
        obs = self.observe()
        quality = self._quality()
        rewards = self._rewards()
        done = self.round % self.cfg.episode_length == 0
        self.former_prio = [j.prio for j in self.core_job]
        self.former_len = [j.rem for j in self.core_job]
        return obs, rewards, quality, done

    # ---- observations (Agent.py:148-300, Auctioneer.py:20-77)
    def acceptor_obs(self, a, c):
        own = int(self.core_owner[c] == a + 1)
        job = self.core_job[c]
        row = [own, job.prio if own else -1, job.rem if own else -1]
        offs = self._offers_to(a + 1, c + 1)
        for o in offs:
            row += [o.price, o.nec_time]
        row += [-2, -2] * (self.O - len(offs))
        return row

    def auctioneer_obs(self, c):
        own = int(self.core_owner[c] == 0)
        job = self.core_job[c]
        row = [own, job.prio if own else -1, job.rem if own else -1]
        offs = self._offers_to(0, c + 1)
        for o in offs:
            row += [o.price, o.nec_time]
        row += [-2, -2] * (self.O - len(offs))
        return row

    def offer_obs(self, a, s):
        row = []
        for c in range(self.C):
            row += [self.core_job[c].prio, self.core_job[c].rem]
        return row + [self.coll[a][s].prio, self.coll[a][s].rem]

    def observe(self):
        acc = [[self.acceptor_obs(a, c) for c in range(self.C)] for a in range(self.N)]
        off = [[self.offer_obs(a, s) for s in range(self.L)] for a in range(self.N)]
        auct = [self.auctioneer_obs(c) for c in range(self.C)]
        return acc, off, auct

    # ---- SchedulingEnv.calculateAverageAcceptionQuality (SchedulingEnvironment.py:174-192)
    def _quality(self):
        qs = []
        for o in self.accepted:
            if o.recipient == 0:
                continue
            c = o.core_id - 1
            q = (o.price / o.nec_time) - (
                (self.former_prio[c] / self.former_len[c]) if self.former_prio[c] != -1 else 0)
            qs.append(q * 10)
        return qs

    # ---- Reward.py:6-89 (free) / :146-212 (fixed)
    def _rewards(self):
        N, C, L = self.N, self.C, self.L
        acc = np.zeros((N, C, 1), dtype=np.int64)
        auct = np.zeros((C,), dtype=np.int64)
        agent = np.zeros((N,), dtype=np.int64)
        term_rev = 0
        if self.cfg.free_prices:
            core_r = np.zeros((N, L, 1), dtype=float)
            price_r = np.zeros((N, L, 1), dtype=float)
            for o in self.accepted:
                diff = o.prio1 - o.price
                if self.cfg.commercial:
                    pr = self.cfg.net_zero_offer_reward if diff == 0 else diff
                else:
                    pr = o.prio1 if diff >= 0 else diff
                price_r[o.offerer - 1][o.queue_pos] = pr
                core_r[o.offerer - 1][o.queue_pos] = o.prio1
            offer_rewards = (core_r, price_r)
        else:
            off_r = np.zeros((N, L, 1), dtype=np.int64)
            for o in self.accepted:
                off_r[o.offerer - 1][o.queue_pos] = o.prio1
            offer_rewards = off_r
        # getAggregatedFixedPricesReward (Reward.py:92-143): the offer reward sums prio1 over the
        # agent's accepted offers, the acceptor reward has no recipient credit
        agg_off = np.zeros((N, 1), dtype=np.int64)
        agg_acc = np.zeros((N, 1), dtype=np.int64)
        for o in self.accepted:
            agg_off[o.offerer - 1][0] += o.prio1
        for c, owner, gen, ts in self.term:
            agg_acc[owner - 1] += gen
            last, tm = ts, 0
            for e in self.liab[c]:
                tm += last - e.round
                last = e.round
                agg_acc[e.offerer - 1] -= round(e.price / e.nec_time * tm)
        self.last_aggregated = (agg_off, agg_acc)
        for c, owner, gen, ts in self.term:
            acc[owner - 1][c] = gen
            if not self.cfg.free_prices:
                agent[owner - 1] += gen
                term_rev += gen
            last, tm = ts, 0
            for e in self.liab[c]:
                tm += last - e.round
                last = e.round
                traded = round(e.price / e.nec_time * tm)
                acc[e.offerer - 1][c] -= traded
                agent[e.offerer - 1] -= traded
                if e.recipient > 0:
                    agent[e.recipient - 1] += traded
                    acc[e.recipient - 1][c] += traded
                if e.recipient == 0:
                    auct[c] = traded
            self.liab[c] = deque()
        return offer_rewards, acc, auct, agent, term_rev

    # ---- aggregated agents: AggregatedAgent (Agent.py:82-134), FullyAggregatedFixPricePPOAgent
    #      (Agent.py:399-464) observations of the current state
    def aggregated_obs(self):
        acc = [[v for c in range(self.C) for v in self.acceptor_obs(a, c)] for a in range(self.N)]
        cores = [v for c in range(self.C) for v in (self.core_job[c].prio, self.core_job[c].rem)]
        off = [cores + [v for j in self.coll[a] for v in (j.prio, j.rem)] for a in range(self.N)]
        fully = [off[a] + acc[a] for a in range(self.N)]  # torch.cat((offer, acceptor)) Agent.py:464
        return acc, off, fully

        # ---- canonical state for comparisons (same fields as ms_state_host)
    def state(self):
        N, C, L = self.N, self.C, self.L
        oc = [[-1] * L for _ in range(N)]
        orc = [[0] * L for _ in range(N)]
        op = [[0] * L for _ in range(N)]
        for o in self.offers:
            oc[o.offerer - 1][o.queue_pos] = o.core_id - 1
            orc[o.offerer - 1][o.queue_pos] = o.recipient
            op[o.offerer - 1][o.queue_pos] = o.price
        liab = []
        for c in range(C):
            liab.append([(e.offerer, e.recipient, e.price, e.nec_time, e.round) for e in reversed(self.liab[c])])
        return dict(
            round=self.round,
            core_owner=list(self.core_owner),
            core_kind=[j.kind for j in self.core_job],
            core_rem=[j.rem for j in self.core_job],
            core_birth=[j.birth for j in self.core_job],
            slot_kind=[[j.kind for j in row] for row in self.coll],
            slot_rem=[[j.rem for j in row] for row in self.coll],
            slot_wait=[[int(j.wait) for j in row] for row in self.coll],
            slot_birth=[[j.birth for j in row] for row in self.coll],
            offer_core=oc, offer_recip=orc, offer_price=op,
            liab=liab,
            mt_state=self.rng.getstate(),
        )


def number_to_nd_action(number, base, dimensionality):
    """numberToNDimensionalAction (Agent.py:644-666), restated."""
    if number < 0 or number >= base ** dimensionality:
        raise ValueError("Illegal Argument")
    out = []
    dim = dimensionality - 1
    n = number
    while len(out) < dimensionality:
        d = n if dim == 0 else n // (base ** dim)
        n -= (base ** dim) * d
        dim -= 1
        out.append(d)
    out.reverse()
    return out
