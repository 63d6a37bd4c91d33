"""Hand-derived known-answer scenarios for the env round (SURVEY.md §8(c) KAT items 2-7 + the spawn edge).

Every expected value below is written out by hand from the reference source (paths relative to
/root/reference/src, cited per scenario), NOT computed by the oracle or the HIP kernel. The
only computation done here is CPython's own `random` module (the pinned RNG, tests/golden/
mt_vectors.json): it supplies the MT19937 state words a scenario starts from and, where the
round draws (a tie-break `random.sample(cands, 1)`, a spawn `random.random()`), which candidate
the draw picks and where the stream index ends. Python float arithmetic is used for one
settlement product to show the value the reference's `round(ratio * T)` sees.

State conventions (the ms_state_host fields, see include/marlsched.h):
  cores: owner (0 = auctioneer), kind (-1 = empty job), rem, birth;
  slots [agent][j]: kind, rem, wait, birth, and the pending offer of the slot made last round
  (offer_core index, recipient, price; offer_core -1 = none); offer IDs are slot order;
  liab[core]: the reference's liabilityList deque in ITS order, newest first (world.py:287
  appendleft), entries (offerer, recipient, price, necessaryTime, round).
Run: python tests/golden/make_kats.py  (writes tests/golden/kats.json)
"""
from __future__ import annotations

import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))

README_JOBS = dict(priorities=[3, 10], lengths=[6, 3], fix_prices=[2, 7], probabilities=[0.8, 0.2])


def mt_state(seed):
    """CPython random.seed(seed) -> (624 words, index)."""
    st = random.Random(seed).getstate()[1]
    return list(st[:624]), st[624]


def rng_at(words, index):
    r = random.Random()
    r.setstate((3, tuple(words) + (index,), None))
    return r


def untemper(y):
    """Inverse of MT19937's output tempering: the state word whose output is y."""
    def undo_right(v, s):
        res = v
        for _ in range(32 // s + 1):
            res = v ^ (res >> s)
        return res & 0xFFFFFFFF

    def undo_left(v, s, m):
        res = v
        for _ in range(32 // s + 1):
            res = v ^ ((res << s) & m)
        return res & 0xFFFFFFFF

    y = undo_right(y, 18)
    y = undo_left(y, 15, 0xEFC60000)
    y = undo_left(y, 7, 0x9D2C5680)
    return undo_right(y, 11)


def empty_state(N, C, L, rnd):
    return dict(round=rnd,
                core_owner=[0] * C, core_kind=[-1] * C, core_rem=[-1] * C, core_birth=[-1] * C,
                slot_kind=[[-1] * L for _ in range(N)], slot_rem=[[-1] * L for _ in range(N)],
                slot_wait=[[0] * L for _ in range(N)], slot_birth=[[-1] * L for _ in range(N)],
                offer_core=[[-1] * L for _ in range(N)], offer_recip=[[0] * L for _ in range(N)],
                offer_price=[[0] * L for _ in range(N)], liab=[[] for _ in range(C)])


def kat_wait_alternation():
    """world.py:406-443 createFixPriceOfferObjectsFromActions: a job offered in round r has
    wait = True, so in round r+1 the else-branch runs whatever the action (no offer, wait = False);
    in round r+2 it is offered again. An action past the last core (coreID C+1, world.py:412-413)
    finds no core: no offer, wait = False. Spawn never fires (L = 1 slot is full: world.py:371-373)."""
    N, C, L = 1, 1, 1
    st = empty_state(N, C, L, 10)
    st["slot_kind"] = [[0]]
    st["slot_rem"] = [[5]]
    st["slot_birth"] = [[9]]
    words, idx = mt_state(101)
    offer = dict(offer_core=[[0]], offer_recip=[[0]], offer_price=[[3]], slot_wait=[[1]])
    none = dict(offer_core=[[-1]], offer_recip=[[0]], offer_price=[[0]], slot_wait=[[0]])
    # the auctioneer rejects explicitly (index O = 1, world.py:388-389): the offer stays unaccepted
    step = lambda off: dict(acc=[[1]], off=[[off]], price=None, auct=[1])
    return dict(
        name="wait_alternation", cites=["world.py:406-443", "world.py:369-376"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, priorities=[4], lengths=[5], fix_prices=[3],
                    probabilities=[1.0]),
        state=st, mt_words=words, mt_index=idx,
        steps=[
            dict(**step(0), expect=dict(state=dict(round=11, slot_kind=[[0]], slot_rem=[[5]], **offer),
                                        # Auctioneer.py:34-77: [owner flag, prio, rem] of the empty core + (price, necT)
                                        obs=dict(auctioneer=[[1, -1, -1, 3, 5]], acceptor=[[[0, -1, -1, -2, -2]]],
                                                 offer=[[[-1, -1, 4, 5]]]),
                                        mt_index=idx)),
            dict(**step(0), expect=dict(state=dict(round=12, **none),
                                        obs=dict(auctioneer=[[1, -1, -1, -2, -2]]))),
            dict(**step(0), expect=dict(state=dict(round=13, **offer))),
            dict(**step(1), expect=dict(state=dict(round=14, **none))),   # wait True -> else branch
            dict(**step(1), expect=dict(state=dict(round=15, **none))),   # coreID 2 does not exist
        ])


def kat_free_price_action0():
    """world.py:445-478 + PPOmodules.py:312-332: the coreChooser's action 0 ("no offer" for the
    policy, priceChooser dummy -5) still maps to coreID 1 in the world, so the job is offered to
    core 1 at price -5; action C maps past the last core: no offer. Next round the hard-coded
    auctioneer sees ratio -5/6 > -1 (HardcodedModules.py:61-76) and accepts it (one candidate:
    random.sample -> one _randbelow(1) draw); the commercial priceChooser reward is
    prio1 - price = 6 - (-5) = 11 (Reward.py:22-35)."""
    N, C, L = 2, 2, 1
    st = empty_state(N, C, L, 5)
    st["slot_kind"] = [[0], [0]]
    st["slot_rem"] = [[6], [6]]
    st["slot_birth"] = [[4], [4]]
    words, idx = mt_state(1234)
    r = rng_at(words, idx)
    assert r._randbelow(1) == 0
    idx_after = r.getstate()[1][624]
    return dict(
        name="free_price_action0", cites=["world.py:445-478", "PPOmodules.py:312-332", "HardcodedModules.py:54-78",
                                          "Reward.py:6-49"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, priorities=[6], lengths=[6], probabilities=[1.0],
                    free_prices=True, commercial=True),
        state=st, mt_words=words, mt_index=idx,
        steps=[
            dict(acc=[[2, 2], [2, 2]], off=[[0], [2]], price=[[-5], [3]], auct=[2, 2],
                 expect=dict(state=dict(round=6, offer_core=[[0], [-1]], offer_recip=[[0], [0]],
                                        offer_price=[[-5], [0]], slot_wait=[[1], [0]]),
                             obs=dict(auctioneer=[[1, -1, -1, -5, 6, -2, -2], [1, -1, -1, -2, -2, -2, -2]]),
                             mt_index=idx)),
            # in-kernel auctioneer (auct = None): core 1 takes offer 1, core 2 has no candidate (no draw)
            dict(acc=[[2, 2], [2, 2]], off=[[2], [2]], price=[[0], [0]], auct=None,
                 expect=dict(state=dict(round=7, core_owner=[1, 0], core_kind=[0, -1], core_rem=[5, -1],
                                        core_birth=[4, -1], slot_kind=[[-1], [0]], slot_rem=[[-1], [6]],
                                        offer_core=[[-1], [-1]], slot_wait=[[0], [0]],
                                        liab=[[[1, 0, -5, 6, 6]], []]),
                             rewards=dict(offer=[[6], [0]], price=[[11], [0]], acceptor=[[0, 0], [0, 0]],
                                          auctioneer=[0, 0], agent=[0, 0]),
                             mt_index=idx_after)),
        ])


def kat_auctioneer_ties():
    """HardcodedModules.py:54-78 + Auctioneer.py:95-102: per core the ratios price/necT of the
    offers addressed to the auctioneer, padded with (-2,-2) -> -1. Core 1: offer-ID order gives
    ratios [2, 2, 1, 2, -1, -1]; max 2 > -1, candidates at positions [0, 1, 3], pick =
    cands[_randbelow(3)] (random.sample(cands, 1), one draw). Core 2: ratios [-1 (price -5 /
    necT 5), -1 (price -1: calculateRewardRatio's -1 rule, :8-9), -1...]: max -1 is not > -1,
    reject, no draw."""
    N, C, L = 3, 2, 2
    st = empty_state(N, C, L, 30)
    #             agent 1 slots 0/1        agent 2 slots 0/1      agent 3 slots 0/1
    st["slot_kind"] = [[0, 0], [0, 0], [0, 0]]
    st["slot_rem"] = [[2, 4], [1, 3], [5, 5]]
    st["slot_birth"] = [[28, 27], [26, 29], [25, 24]]
    st["slot_wait"] = [[1, 1], [1, 1], [1, 1]]
    st["offer_core"] = [[0, 0], [0, 0], [1, 1]]
    st["offer_recip"] = [[0, 0], [0, 0], [0, 0]]
    st["offer_price"] = [[4, 8], [1, 6], [-5, -1]]
    words, idx = mt_state(779)  # _randbelow(3) = 2: the non-adjacent tie at position 3
    r = rng_at(words, idx)
    j = r._randbelow(3)
    idx_after = r.getstate()[1][624]
    pick = [0, 1, 3][j]
    # outcome per picked position (slot index = position: offer IDs are slot order), by hand:
    outcomes = {
        0: dict(owner=1, rem=1, birth=28, price=4, nec=2, slot_kind=[[-1, 0], [0, 0], [0, 0]],
                offer=[[12, 0], [0, 0], [0, 0]], price_r=[[8, 0], [0, 0], [0, 0]]),
        1: dict(owner=1, rem=3, birth=27, price=8, nec=4, slot_kind=[[0, -1], [0, 0], [0, 0]],
                offer=[[0, 12], [0, 0], [0, 0]], price_r=[[0, 4], [0, 0], [0, 0]]),
        3: dict(owner=2, rem=2, birth=29, price=6, nec=3, slot_kind=[[0, 0], [0, -1], [0, 0]],
                offer=[[0, 0], [0, 12], [0, 0]], price_r=[[0, 0], [0, 6], [0, 0]]),
    }[pick]
    o = outcomes
    return dict(
        name="auctioneer_ties", cites=["HardcodedModules.py:5-13", "HardcodedModules.py:54-78", "Auctioneer.py:95-102",
                                       "world.py:378-389", "Reward.py:22-35"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, priorities=[12], lengths=[6], probabilities=[1.0],
                    free_prices=True, commercial=True),
        state=st, mt_words=words, mt_index=idx, note="CPython _randbelow(3) = %d -> position %d" % (j, pick),
        steps=[
            dict(acc=[[6, 6]] * 3, off=[[2, 2]] * 3, price=[[0, 0]] * 3, auct=None,
                 expect=dict(state=dict(round=31, core_owner=[o["owner"], 0], core_kind=[0, -1],
                                        core_rem=[o["rem"], -1], core_birth=[o["birth"], -1],
                                        slot_kind=o["slot_kind"], slot_wait=[[0, 0]] * 3,
                                        offer_core=[[-1, -1]] * 3,
                                        liab=[[[o["owner"], 0, o["price"], o["nec"], 30]], []]),
                             rewards=dict(offer=o["offer"], price=o["price_r"], acceptor=[[0, 0]] * 3,
                                          auctioneer=[0, 0], agent=[0, 0, 0]),
                             obs=dict(auctioneer=[[0, -1, -1] + [-2] * 12, [1, -1, -1] + [-2] * 12]),
                             mt_index=idx_after)),
        ])


def kat_spawn_edge():
    """world.py:220-222 + Agent.py:50-70: accProbabilities [0.5, 0.9] (sum < 1). A draw u >= 0.9
    matches no kind; the reference then reads the unassigned local `randomIndex` and raises
    UnboundLocalError. The build clamps to the last kind and sets MS_FLAG_SPAWN_EDGE (0x08)
    (DESIGN.md §8). The next draw u < 0.9 picks kind 1 normally. random() = (a>>5 * 2^26 + b>>6) / 2^53
    of two tempered words a, b: the state words are crafted as untemper(a), untemper(b)."""
    N, C, L = 1, 1, 2
    st = empty_state(N, C, L, 0)
    words, _ = mt_state(7)
    idx = 100
    words[100], words[101] = untemper(0xF0000000), untemper(0x12345678)   # u = 0.9375...
    words[102], words[103] = untemper(0xE0000000), untemper(0x00000000)   # u = 0.875
    r = rng_at(words, idx)
    u1, u2 = r.random(), r.random()
    assert u1 >= 0.9 and 0.5 <= u2 < 0.9
    return dict(
        name="spawn_edge", cites=["world.py:220-222", "Agent.py:50-70", "world.py:369-376"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, probabilities=[0.5, 0.4], **{
            k: v for k, v in README_JOBS.items() if k != "probabilities"}),
        state=st, mt_words=words, mt_index=idx, note="u1 = %r, u2 = %r" % (u1, u2),
        steps=[
            dict(acc=[[2]], off=[[1, 1]], price=None, auct=[2],
                 expect=dict(state=dict(round=1, slot_kind=[[1, -1]], slot_rem=[[3, -1]], slot_birth=[[0, -1]]),
                             flags_set=0x08, mt_index=102)),
            dict(acc=[[2]], off=[[1, 1]], price=None, auct=[2],
                 expect=dict(state=dict(round=2, slot_kind=[[1, 1]], slot_rem=[[3, 3]], slot_birth=[[0, 1]]),
                             flags_set=0x08, mt_index=104)),   # per-env flags are sticky
        ])


def kat_self_offer_first_empty():
    """world.py:261-293 + :123-141 + :391-404: agent 1 owns both cores (X on core 1, Y on core 2)
    and has slots [empty, A, empty]; A is offered to core 2 (a self-offer: recipient = core owner =
    agent 1), agent 2's B to core 1. Agent 1's acceptors take both, executed in agent order then
    core order: core 1 first -> B on core 1 (owner := B's owner 2), X into agent 1's first empty
    slot = slot 0; then core 2 -> A leaves slot 1, A on core 2, Y into the first empty slot, now
    slot 1. Result [X, Y, empty]; the opposite order would give [Y, X, empty]."""
    N, C, L = 2, 2, 3
    st = empty_state(N, C, L, 40)
    st.update(core_owner=[1, 1], core_kind=[0, 1], core_rem=[4, 3], core_birth=[35, 36])
    st["slot_kind"] = [[-1, 0, -1], [1, 0, 0]]
    st["slot_rem"] = [[-1, 6, -1], [3, 6, 6]]
    st["slot_birth"] = [[-1, 38, -1], [39, 37, 39]]
    st["slot_wait"] = [[0, 1, 0], [1, 0, 0]]
    st["offer_core"] = [[-1, 1, -1], [0, -1, -1]]
    st["offer_recip"] = [[0, 1, 0], [1, 0, 0]]
    st["offer_price"] = [[0, 2, 0], [7, 0, 0]]   # fixPrices[kind]: A kind 0 -> 2, B kind 1 -> 7
    words, idx = mt_state(55)
    return dict(
        name="self_offer_first_empty", cites=["world.py:123-141", "world.py:261-293", "world.py:391-404",
                                              "Reward.py:164-170"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, **README_JOBS),
        state=st, mt_words=words, mt_index=idx,
        steps=[
            dict(acc=[[0, 0], [6, 6]], off=[[2, 2, 2], [2, 2, 2]], price=None, auct=[6, 6],
                 expect=dict(state=dict(round=41, core_owner=[2, 1], core_kind=[1, 0], core_rem=[2, 5],
                                        core_birth=[39, 38],
                                        slot_kind=[[0, 1, -1], [-1, 0, 0]], slot_rem=[[4, 3, -1], [-1, 6, 6]],
                                        slot_birth=[[35, 36, -1], [-1, 37, 39]], slot_wait=[[0, 0, 0], [0, 0, 0]],
                                        offer_core=[[-1, -1, -1], [-1, -1, -1]],
                                        liab=[[[2, 1, 7, 3, 40]], [[1, 1, 2, 6, 40]]]),
                             rewards=dict(offer=[[0, 3, 0], [10, 0, 0]], acceptor=[[0, 0], [0, 0]], auctioneer=[0, 0],
                                          agent=[0, 0]),
                             # Agent.py:167-212 / 271-300 on the new state
                             obs=dict(acceptor=[[[0, -1, -1] + [-2] * 12, [1, 3, 5] + [-2] * 12],
                                                [[1, 10, 2] + [-2] * 12, [0, -1, -1] + [-2] * 12]],
                                      offer=[[[10, 2, 3, 5, 3, 4], [10, 2, 3, 5, 10, 3], [10, 2, 3, 5, -1, -1]],
                                             [[10, 2, 3, 5, -1, -1], [10, 2, 3, 5, 3, 6], [10, 2, 3, 5, 3, 6]]]),
                             mt_index=idx)),
        ])


def kat_mixed_chain():
    """Reward.py:187-210 (fixed prices): core 1's job (prio 10) ends this round (TS = round+1 = 21).
    The chain, newest first: e1 (1 -> auctioneer, price 5, necT 4, round 19), e2 (2 -> agent 1,
    price 2, necT 6, round 17), e3 (1 -> auctioneer, price 7, necT 5, round 12). Walk:
      acc[1][1] = 10, agent[1] = 10
      e1: T = 21-19 = 2, round(1.25*2 = 2.5) = 2 (half-even): acc[1] -= 2, agent[1] -= 2, auct = 2
      e2: T = 2 + 2 = 4, round(0.333..*4) = 1: acc[2] -= 1, agent[2] -= 1; recipient 1: acc[1] += 1, agent[1] += 1
      e3: T = 4 + 5 = 9, round(1.4*9) = 13: acc[1] -= 13, agent[1] -= 13, auct = 13 (the last
          auctioneer entry visited overwrites, :207-208)
    -> acceptor [[-4], [-1]], agent [-4, -1], auctioneer [13]; the chain is reset (:210).
    Then agent 1 (no core, 2 free slots) spawns one job from random() (kind 0 if u < 0.8)."""
    N, C, L = 2, 1, 2
    st = empty_state(N, C, L, 20)
    st.update(core_owner=[1], core_kind=[1], core_rem=[1], core_birth=[14])
    st["slot_kind"] = [[-1, -1], [0, 0]]
    st["slot_rem"] = [[-1, -1], [6, 6]]
    st["slot_birth"] = [[-1, -1], [19, 19]]
    st["liab"] = [[[1, 0, 5, 4, 19], [2, 1, 2, 6, 17], [1, 0, 7, 5, 12]]]
    assert round(5 / 4 * 2) == 2 and round(2 / 6 * 4) == 1 and round(7 / 5 * 9) == 13
    words, idx = mt_state(4242)
    r = rng_at(words, idx)
    u = r.random()
    kind = 0 if u < 0.8 else 1
    return dict(
        name="mixed_chain", cites=["Reward.py:146-212", "world.py:336-367", "world.py:369-376"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, **README_JOBS),
        state=st, mt_words=words, mt_index=idx, note="spawn u = %r -> kind %d" % (u, kind),
        steps=[
            dict(acc=[[4], [4]], off=[[1, 1], [1, 1]], price=None, auct=[4],
                 expect=dict(state=dict(round=21, core_owner=[0], core_kind=[-1], core_rem=[-1], liab=[[]],
                                        slot_kind=[[kind, -1], [0, 0]], slot_rem=[[[6, 3][kind], -1], [6, 6]],
                                        slot_birth=[[20, -1], [19, 19]]),
                             rewards=dict(acceptor=[[-4], [-1]], agent=[-4, -1], auctioneer=[13],
                                          offer=[[0, 0], [0, 0]]),
                             termination_revenue=10, mt_index=r.getstate()[1][624])),
        ])


def kat_settlement_double_product():
    """Reward.py:200-201 (free prices): traded = round(fl(7/6) * 105) = round(122.50000000000001) =
    123, not the exact-rational 122.5 -> 122 (SURVEY.md §8(c) KAT 1)."""
    N, C, L = 2, 1, 1
    st = empty_state(N, C, L, 104)
    st.update(core_owner=[1], core_kind=[0], core_rem=[1], core_birth=[0])
    st["liab"] = [[[1, 0, 7, 6, 0]]]
    assert round(7 / 6 * 105) == 123
    words, idx = mt_state(3)
    r = rng_at(words, idx)
    r.random(), r.random()  # both agents spawn one job (one kind: any u), agent 1 after losing its core
    return dict(
        name="settlement_double_product", cites=["Reward.py:59-82"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, priorities=[12], lengths=[6], probabilities=[1.0],
                    free_prices=True, commercial=True),
        state=st, mt_words=words, mt_index=idx,
        steps=[
            dict(acc=[[2], [2]], off=[[1], [1]], price=[[-5], [-5]], auct=[2],
                 expect=dict(state=dict(round=105, core_owner=[0], liab=[[]], slot_kind=[[0], [0]]),
                             rewards=dict(acceptor=[[12 - 123], [0]], agent=[-123, 0], auctioneer=[123]),
                             mt_index=r.getstate()[1][624])),
        ])


def kat_net_zero_offer_reward():
    """Reward.py:22-35 (commercial free prices): the priceChooser reward of an accepted offer whose
    price equals the job's priority is env.netZeroOfferReward (0.5, SchedulingEnvironment.py's
    default) instead of prio1 - price = 0; the coreChooser reward is prio1. The auctioneer (explicit
    action: position 0 of core 1) takes agent 1's offer (price 6 = prio 6); the job goes onto core 1
    (world.py:261-293) and ticks 6 -> 5 (world.py:336-367). Agent 1 (owns core 1, no free slot
    left after... its slot was freed, 1 + 1 > 1) does not spawn; agent 2 (0 + 1 <= 1) draws one
    random() for its job (one kind: any u)."""
    N, C, L = 2, 2, 1
    st = empty_state(N, C, L, 5)
    st["slot_kind"] = [[0], [-1]]
    st["slot_rem"] = [[6], [-1]]
    st["slot_birth"] = [[4], [-1]]
    st["slot_wait"] = [[1], [0]]
    st["offer_core"] = [[0], [-1]]
    st["offer_recip"] = [[0], [0]]
    st["offer_price"] = [[6], [0]]
    words, idx = mt_state(2024)
    r = rng_at(words, idx)
    r.random()
    return dict(
        name="net_zero_offer_reward", cites=["Reward.py:22-35", "world.py:261-293", "world.py:369-376"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, priorities=[6], lengths=[6], probabilities=[1.0],
                    free_prices=True, commercial=True),
        state=st, mt_words=words, mt_index=idx,
        steps=[
            dict(acc=[[2, 2], [2, 2]], off=[[2], [2]], price=[[0], [0]], auct=[0, 2],
                 expect=dict(state=dict(round=6, core_owner=[1, 0], core_kind=[0, -1], core_rem=[5, -1],
                                        core_birth=[4, -1], slot_kind=[[-1], [0]], slot_rem=[[-1], [6]],
                                        slot_birth=[[-1], [5]], slot_wait=[[0], [0]], offer_core=[[-1], [-1]],
                                        liab=[[[1, 0, 6, 6, 5]], []]),
                             rewards=dict(offer=[[6], [0]], price=[[0.5], [0]], acceptor=[[0, 0], [0, 0]],
                                          auctioneer=[0, 0], agent=[0, 0]),
                             mt_index=r.getstate()[1][624])),
        ])


def kat_noncommercial_price_reward():
    """Reward.py:36-49 (non-commercial free prices): priceChooser reward = prio1 if prio1 - price >= 0,
    else prio1 - price (negative). Agent 1 offered its prio-6 job to core 1 at price 8 (-> 6 - 8 =
    -2), agent 2 its prio-8 job to core 2 at price 3 (-> 8). The auctioneer takes both (explicit
    actions, position 0 of each core); both agents then own a core and have no free slot: no spawn,
    no draw."""
    N, C, L = 2, 2, 1
    st = empty_state(N, C, L, 7)
    st["slot_kind"] = [[0], [1]]
    st["slot_rem"] = [[6], [6]]
    st["slot_birth"] = [[6], [5]]
    st["slot_wait"] = [[1], [1]]
    st["offer_core"] = [[0], [1]]
    st["offer_recip"] = [[0], [0]]
    st["offer_price"] = [[8], [3]]
    words, idx = mt_state(77)
    return dict(
        name="noncommercial_price_reward", cites=["Reward.py:36-49", "world.py:261-293"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, priorities=[6, 8], lengths=[6, 6],
                    probabilities=[0.5, 0.5], free_prices=True, commercial=False),
        state=st, mt_words=words, mt_index=idx,
        steps=[
            dict(acc=[[2, 2], [2, 2]], off=[[2], [2]], price=[[0], [0]], auct=[0, 0],
                 expect=dict(state=dict(round=8, core_owner=[1, 2], core_kind=[0, 1], core_rem=[5, 5],
                                        core_birth=[6, 5], slot_kind=[[-1], [-1]], offer_core=[[-1], [-1]],
                                        liab=[[[1, 0, 8, 6, 7]], [[2, 0, 3, 6, 7]]]),
                             rewards=dict(offer=[[6], [8]], price=[[-2], [8]], acceptor=[[0, 0], [0, 0]],
                                          auctioneer=[0, 0], agent=[0, 0]),
                             mt_index=idx)),
        ])


def kat_two_jobs_first_empty():
    """world.py:369-376 + Agent.py:50-70 with newJobsPerRoundPerAgent = 2: agent 1 (no core, slots
    [A, -, B, -]: 0 + 2 <= 2 free) draws two random() in a row; the kind of each is the first i with
    u < accProbabilities[i] ([0.5, 1.0]) and it goes into the first empty slot (world.py:123-133):
    slot 1, then slot 3. Agent 2 (slots [C, D, E, -]: 0 + 2 > 1 free) spawns nothing. No offers:
    action 1 maps to coreID 2, which does not exist (world.py:412-413)."""
    N, C, L = 2, 1, 4
    st = empty_state(N, C, L, 30)
    st["slot_kind"] = [[0, -1, 1, -1], [1, 0, 1, -1]]
    st["slot_rem"] = [[4, -1, 2, -1], [2, 4, 1, -1]]
    st["slot_birth"] = [[28, -1, 29, -1], [27, 26, 29, -1]]
    words, idx = mt_state(31337)
    r = rng_at(words, idx)
    u1, u2 = r.random(), r.random()
    k1, k2 = (0 if u1 < 0.5 else 1), (0 if u2 < 0.5 else 1)
    lens = [4, 2]
    return dict(
        name="two_jobs_first_empty", cites=["world.py:369-376", "Agent.py:50-70", "world.py:123-133"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, priorities=[4, 8], lengths=lens, fix_prices=[2, 4],
                    probabilities=[0.5, 0.5], new_jobs=2),
        state=st, mt_words=words, mt_index=idx, note="u1 = %r -> kind %d, u2 = %r -> kind %d" % (u1, k1, u2, k2),
        steps=[
            dict(acc=[[8], [8]], off=[[1] * 4, [1] * 4], price=None, auct=[8],
                 expect=dict(state=dict(round=31, slot_kind=[[0, k1, 1, k2], [1, 0, 1, -1]],
                                        slot_rem=[[4, lens[k1], 2, lens[k2]], [2, 4, 1, -1]],
                                        slot_birth=[[28, 30, 29, 30], [27, 26, 29, -1]],
                                        slot_wait=[[0] * 4, [0] * 4], offer_core=[[-1] * 4, [-1] * 4]),
                             mt_index=r.getstate()[1][624])),
        ])


def kat_hardcoded_agent_ties():
    """HardcodedModules.py:16-45 (acceptor) and :81-109 (offerer) acting inside the round (the
    HardcodedFixPriceEnvironment loop, SchedulingEnvironment.py:439-456), their random.sample draws
    in getActions order (per agent: offer slots, then acceptor cores), then the auctioneer's (none:
    it owns no core), then spawn. Both cores hold (prio 4, rem 4): every offerer sees core ratios
    [1, 1], a tie -> cands[_randbelow(2)] per slot (empty slots draw too). Agent 1's acceptor of
    core 1 (own ratio 1) sees agent 2's two offers (4, 2), (4, 2): ratios [2, 2, -1, ...], a tie ->
    _randbelow(2) picks which one it takes. Agent 2's acceptor of core 2 (own ratio 1) sees agent
    1's offer (4, 1): ratio 4 > 1, one candidate (_randbelow(1)). Executions in agent order: agent 2's
    picked job (prio 8, rem 2) onto core 1 (owner 2), the old core-1 job to agent 1's first empty
    slot (slot 1); agent 1's (prio 8, rem 1) onto core 2 (owner 1), the old core-2 job to agent 2's
    first empty slot (the picked one's). Tick: core 1 -> rem 1; core 2 ends (TS 51): acc[1][2] = 8,
    agent[1] += 8; chain (1 -> 2, price 4, necT 1, round 50): T = 1, traded = 4 -> acc[1][2] = 4,
    agent[1] = 4, acc[2][2] = agent[2] = 4. Offers then follow the slot draws (core index ->
    recipient = that core's owner after the tick: core 1 -> 2, core 2 -> auctioneer); agent 1 (no
    core, 2 free slots) spawns one job into slot 0; agent 2 (1 core, 1 free slot) does not."""
    N, C, L = 2, 2, 3
    st = empty_state(N, C, L, 50)
    st.update(core_owner=[1, 2], core_kind=[0, 0], core_rem=[4, 4], core_birth=[45, 46])
    st["slot_kind"] = [[1, -1, -1], [1, 1, -1]]
    st["slot_rem"] = [[1, -1, -1], [2, 2, -1]]
    st["slot_birth"] = [[49, -1, -1], [47, 48, -1]]
    st["slot_wait"] = [[1, 0, 0], [1, 1, 0]]
    st["offer_core"] = [[1, -1, -1], [0, 0, -1]]
    st["offer_recip"] = [[2, 0, 0], [1, 1, 0]]
    st["offer_price"] = [[4, 0, 0], [4, 4, 0]]
    words, idx = mt_state(9001)
    r = rng_at(words, idx)
    a1s = [r._randbelow(2) for _ in range(L)]   # agent 1's offerers (slots 0, 1, 2)
    p = r._randbelow(2)                         # agent 1's acceptor of core 1: which of agent 2's offers
    a2s = [r._randbelow(2) for _ in range(L)]   # agent 2's offerers
    assert r._randbelow(1) == 0                 # agent 2's acceptor of core 2: one candidate
    u = r.random()                              # agent 1's spawn
    kind = 0 if u < 0.5 else 1
    owner_after = [2, 0]                        # core owners after the tick
    # agent 1: slot 0 = spawned job; slot 1 = old core-1 job (kind 0, rem 4, birth 45), offered per a1s[1]
    # agent 2: slot p = old core-2 job (kind 0, rem 4, birth 46), offered per a2s[p]; slot 1-p = the
    # unaccepted offer's job (wait -> else branch: no offer, wait False); slot 2 empty
    a2_kind, a2_rem, a2_birth = [0, 0, -1], [0, 0, -1], [0, 0, -1]
    a2_kind[p], a2_rem[p], a2_birth[p] = 0, 4, 46
    a2_kind[1 - p], a2_rem[1 - p], a2_birth[1 - p] = 1, 2, [47, 48][1 - p]
    a2_off, a2_rcp, a2_pr, a2_wait = [-1, -1, -1], [0, 0, 0], [0, 0, 0], [0, 0, 0]
    a2_off[p], a2_rcp[p], a2_pr[p], a2_wait[p] = a2s[p], owner_after[a2s[p]], 2, 1
    return dict(
        name="hardcoded_agent_ties", cites=["HardcodedModules.py:5-45", "HardcodedModules.py:81-109",
                                            "SchedulingEnvironment.py:439-456", "world.py:261-293",
                                            "world.py:336-367", "Reward.py:146-212", "world.py:406-443"],
        device_only="the C oracle takes actions from the caller; the in-kernel hard-coded agents are "
                    "checked here and in tests/test_hardcoded_gpu.py against oracle/pyref.py",
        config=dict(n_agents=N, n_cores=C, collection_length=L, priorities=[4, 8], lengths=[4, 2], fix_prices=[2, 4],
                    probabilities=[0.5, 0.5]),
        state=st, mt_words=words, mt_index=idx,
        note="offerer draws agent 1 %s, agent 2 %s; acceptor tie -> offer position %d; spawn u = %r -> kind %d"
             % (a1s, a2s, p, u, kind),
        steps=[
            dict(acc=None, off=None, price=None, auct=None,
                 expect=dict(state=dict(round=51, core_owner=[2, 0], core_kind=[1, -1], core_rem=[1, -1],
                                        core_birth=[[47, 48][p], -1],
                                        slot_kind=[[kind, 0, -1], a2_kind], slot_rem=[[[4, 2][kind], 4, -1], a2_rem],
                                        slot_birth=[[50, 45, -1], a2_birth], slot_wait=[[0, 1, 0], a2_wait],
                                        offer_core=[[-1, a1s[1], -1], a2_off],
                                        offer_recip=[[0, owner_after[a1s[1]], 0], a2_rcp],
                                        offer_price=[[0, 2, 0], a2_pr],
                                        liab=[[[2, 1, 4, 2, 50]], []]),
                             rewards=dict(offer=[[8, 0, 0], [8 if p == 0 else 0, 8 if p == 1 else 0, 0]],
                                          acceptor=[[0, 4], [0, 4]], auctioneer=[0, 0], agent=[4, 4]),
                             mt_index=r.getstate()[1][624])),
        ])


def kat_liability_overflow():
    """The liability chain (world.py:238, 287: an unbounded deque in the reference) is held in
    liability_cap entries per core here. A third accepted offer on a core whose chain already holds
    liability_cap = 2 entries is dropped and sets MS_FLAG_LIABILITY_OVERFLOW (0x01);
    the flag is fatal: the next ms_env_step returns MS_EOVERFLOW (75) without launching. The
    execution itself follows world.py:261-293 (agent 2's job onto core 1, the old job to agent 1's
    first empty slot) and the offer reward Reward.py:164-170."""
    N, C, L = 2, 1, 1
    st = empty_state(N, C, L, 13)
    st.update(core_owner=[1], core_kind=[0], core_rem=[5], core_birth=[10])
    st["slot_kind"] = [[-1], [0]]
    st["slot_rem"] = [[-1], [6]]
    st["slot_birth"] = [[-1], [12]]
    st["slot_wait"] = [[0], [1]]
    st["offer_core"] = [[-1], [0]]
    st["offer_recip"] = [[0], [1]]
    st["offer_price"] = [[0], [2]]
    st["liab"] = [[[1, 2, 2, 6, 12], [2, 0, 2, 6, 11]]]
    words, idx = mt_state(5)
    return dict(
        name="liability_overflow", cites=["world.py:238", "world.py:261-293", "Reward.py:164-170"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, liability_cap=2, **README_JOBS),
        state=st, mt_words=words, mt_index=idx,
        steps=[
            dict(acc=[[0], [2]], off=[[1], [1]], price=None, auct=[2],
                 expect=dict(state=dict(round=14, core_owner=[2], core_kind=[0], core_rem=[5], core_birth=[12],
                                        slot_kind=[[0], [-1]], slot_rem=[[5], [-1]], slot_birth=[[10], [-1]],
                                        liab=[[[1, 2, 2, 6, 12], [2, 0, 2, 6, 11]]]),
                             rewards=dict(offer=[[0], [3]], acceptor=[[0], [0]], auctioneer=[0], agent=[0, 0]),
                             flags_set=0x01, mt_index=idx)),
            dict(acc=[[1], [1]], off=[[1], [1]], price=None, auct=[1], expect=dict(error=75)),
        ])


def kat_aggregated_chain_rewards():
    """Reward.py:92-143 getAggregatedFixedPricesReward, written out by hand next to the divided
    Reward.py:146-212 of the same round. Round 10, fixed prices. Core 1 (agent 1, prio 10, one round
    left) ends this round, TS = 11; its chain newest first: e1 (1 -> agent 2, price 7, necT 3,
    round 8), e2 (2 -> auctioneer, price 2, necT 6, round 4). Agent 3's pending offer (slot 0, kind 0,
    rem 5, to core 2 held by the auctioneer, price fixPrices[0] = 2) is accepted by the auctioneer.
      aggregated offer (:95-101): offerRewards[offerer] += prio1 -> agent 3: 3
      termination (:121-122): acceptorRewards[1] += 10, agentReward[1] += 10
      e1: T = 11-8 = 3, round(fl(7/3)*3) = round(7.000000000000001) = 7 (:130-131):
          acceptorRewards[1] -= 7, agentReward[1] -= 7; recipient 2 > 0: agentReward[2] += 7 only
          (:136-137: no acceptor credit, unlike the divided :203-205)
      e2: T = 3 + (8-4) = 7, round(fl(2/6)*7) = round(2.333...) = 2: acceptorRewards[2] -= 2,
          agentReward[2] -= 2; recipient 0: auctioneerReward[1] = 2
    -> aggregated acceptor [3, -2, 0], offer [0, 0, 3], agent [3, 5, 0], auctioneer [2, 0].
    The divided acceptor rewards of the same round credit the recipient: [[3, 0], [5, 0], [0, 0]].
    Spawn: agent 1 (no core, one free slot) draws one job; agent 2 (full) and agent 3 (owns core 2,
    one free slot: 1 + 1 > 1) do not."""
    N, C, L = 3, 2, 2
    st = empty_state(N, C, L, 10)
    st.update(core_owner=[1, 0], core_kind=[1, -1], core_rem=[1, -1], core_birth=[7, -1])
    st["slot_kind"] = [[0, -1], [1, 0], [0, 1]]
    st["slot_rem"] = [[6, -1], [3, 6], [5, 3]]
    st["slot_birth"] = [[9, -1], [6, 9], [9, 5]]
    st["slot_wait"] = [[0, 0], [0, 0], [1, 0]]
    st["offer_core"] = [[-1, -1], [-1, -1], [1, -1]]
    st["offer_recip"] = [[0, 0], [0, 0], [0, 0]]
    st["offer_price"] = [[0, 0], [0, 0], [2, 0]]
    st["liab"] = [[[1, 2, 7, 3, 8], [2, 0, 2, 6, 4]], []]
    assert round(7 / 3 * 3) == 7 and round(2 / 6 * 7) == 2
    words, idx = mt_state(2718)
    r = rng_at(words, idx)
    u = r.random()
    kind = 0 if u < 0.8 else 1
    return dict(
        name="aggregated_chain_rewards", cites=["Reward.py:92-143", "Reward.py:146-212", "world.py:378-389"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, **README_JOBS),
        state=st, mt_words=words, mt_index=idx, note="spawn u = %r -> kind %d" % (u, kind),
        steps=[
            dict(acc=[[6, 6]] * 3, off=[[2, 2]] * 3, price=None, auct=[6, 0],
                 expect=dict(state=dict(round=11, core_owner=[0, 3], core_kind=[-1, 0], core_rem=[-1, 4],
                                        core_birth=[-1, 9],
                                        slot_kind=[[0, kind], [1, 0], [-1, 1]],
                                        slot_rem=[[6, [6, 3][kind]], [3, 6], [-1, 3]],
                                        slot_birth=[[9, 10], [6, 9], [-1, 5]], slot_wait=[[0, 0]] * 3,
                                        offer_core=[[-1, -1]] * 3, liab=[[], [[3, 0, 2, 5, 10]]]),
                             rewards=dict(aggregated_offer=[0, 0, 3], aggregated_acceptor=[3, -2, 0],
                                          agent=[3, 5, 0], auctioneer=[2, 0],
                                          acceptor=[[3, 0], [5, 0], [0, 0]], offer=[[0, 0], [0, 0], [3, 0]]),
                             termination_revenue=10, mt_index=r.getstate()[1][624])),
        ])


def kat_acception_quality():
    """SchedulingEnvironment.py:174-192 calculateAverageAcceptionQuality: for every accepted offer
    whose recipient is an agent, 10 * (offeredReward / necessaryTime - formerCorePrio /
    formerCoreLength), the former values being the core's job when the previous step ended
    (:64-66: after that round's tick, i.e. the state this round starts from; 0 for an empty core).
    Round 20, fixed prices, N = 2, C = 2, L = 3. Core 1: agent 1, prio 3, rem 4; core 2: agent 2,
    prio 10, rem 2. Offer IDs (slot order): 1 = agent 1 slot 0 (kind 1, rem 3, price 7) to core 2
    (recipient 2); 2 = agent 2 slot 0 (kind 0, rem 6, price 2) and 3 = agent 2 slot 1 (kind 1,
    rem 3, price 7) to core 1 (recipient 1). Agent 1's core-1 acceptor takes index 1 = offer 3, agent
    2's core-2 acceptor index 0 = offer 1; executions in agent order (world.py:391-404):
      offer 3: 10 * (7/3 - 3/4)  = 10 * (2.3333333333333335 - 0.75)
      offer 1: 10 * (7/3 - 10/2) = 10 * (2.3333333333333335 - 5.0)
    the round's value is statistics.mean of the two, amount 2. Each old core job goes to its
    owner's first empty slot (agent 1 slot 1, agent 2 slot 1); agent 1 then spawns into slot 0."""
    import statistics

    N, C, L = 2, 2, 3
    st = empty_state(N, C, L, 20)
    st.update(core_owner=[1, 2], core_kind=[0, 1], core_rem=[4, 2], core_birth=[15, 17])
    st["slot_kind"] = [[1, -1, -1], [0, 1, -1]]
    st["slot_rem"] = [[3, -1, -1], [6, 3, -1]]
    st["slot_birth"] = [[16, -1, -1], [19, 18, -1]]
    st["slot_wait"] = [[1, 0, 0], [1, 1, 0]]
    st["offer_core"] = [[1, -1, -1], [0, 0, -1]]
    st["offer_recip"] = [[2, 0, 0], [1, 1, 0]]
    st["offer_price"] = [[7, 0, 0], [2, 7, 0]]
    q3 = (7 / 3 - 3 / 4) * 10
    q1 = (7 / 3 - 10 / 2) * 10
    words, idx = mt_state(31415)
    r = rng_at(words, idx)
    u = r.random()
    kind = 0 if u < 0.8 else 1
    return dict(
        name="acception_quality", cites=["SchedulingEnvironment.py:64-66", "SchedulingEnvironment.py:174-192",
                                         "world.py:391-404", "world.py:123-133"],
        config=dict(n_agents=N, n_cores=C, collection_length=L, **README_JOBS),
        state=st, mt_words=words, mt_index=idx, note="spawn u = %r -> kind %d" % (u, kind),
        steps=[
            dict(acc=[[1, 6], [6, 0]], off=[[2, 2, 2], [2, 2, 2]], price=None, auct=[6, 6],
                 expect=dict(state=dict(round=21, core_owner=[2, 1], core_kind=[1, 1], core_rem=[2, 2],
                                        core_birth=[18, 16],
                                        slot_kind=[[kind, 0, -1], [0, 1, -1]],
                                        slot_rem=[[[6, 3][kind], 4, -1], [6, 2, -1]],
                                        slot_birth=[[20, 15, -1], [19, 17, -1]], slot_wait=[[0, 0, 0]] * 2,
                                        offer_core=[[-1, -1, -1]] * 2,
                                        liab=[[[2, 1, 7, 3, 20]], [[1, 2, 7, 3, 20]]]),
                             rewards=dict(offer=[[10, 0, 0], [0, 10, 0]], acceptor=[[0, 0], [0, 0]],
                                          agent=[0, 0], auctioneer=[0, 0]),
                             quality=[q3, q1], quality_mean=statistics.mean([q3, q1]),
                             mt_index=r.getstate()[1][624])),
        ])


def codec_cases():
    """numberToNDimensionalAction (Agent.py:644-666) as the aggregated agents use it (Agent.py:373-380:
    acceptor number -> C digits in base O+1, offer number -> L digits in base C+1; fully aggregated
    Agent.py:469-473: acceptor = a // (C+1)^L, offer = a % (C+1)^L), written out by hand for N = C = L
    = 2 (O = 4: bases 5 and 3). The loop takes the most significant digit first and reverses, so
    digit i (action of core / slot i) is the base^i digit:
      acceptor 13: dimension 1: 13 // 5 = 2, rest 3; dimension 0: 3 -> [2, 3] reversed = [3, 2]
      offer 7: 7 // 3 = 2, rest 1 -> [1, 2]
      fully 124 = 13 * 9 + 7 -> acceptor 13, offer 7
    A number outside [0, base^dim) raises ValueError("Illegal Argument") (:651-652)."""
    return dict(
        name="codec", cites=["Agent.py:644-666", "Agent.py:373-380", "Agent.py:469-473"],
        config=dict(n_agents=2, n_cores=2, collection_length=2, **README_JOBS),
        plain=[dict(number=0, base=5, dim=2, digits=[0, 0]), dict(number=13, base=5, dim=2, digits=[3, 2]),
               dict(number=24, base=5, dim=2, digits=[4, 4]), dict(number=5, base=5, dim=2, digits=[0, 1]),
               dict(number=7, base=3, dim=2, digits=[1, 2]), dict(number=8, base=3, dim=2, digits=[2, 2]),
               dict(number=26, base=3, dim=3, digits=[2, 2, 2]), dict(number=4, base=5, dim=1, digits=[4]),
               dict(number=0, base=1, dim=3, digits=[0, 0, 0]),
               dict(number=25, base=5, dim=2, error="ValueError"), dict(number=-1, base=5, dim=2, error="ValueError"),
               dict(number=9, base=3, dim=2, error="ValueError"), dict(number=1, base=1, dim=3, error="ValueError")],
        # device form (ms_decode_aggregated): per agent (acceptor number, offer number) -> actions. In
        # the reference one illegal number raises out of getActions (Agent.py:368-382), so the agent
        # takes no action at all: the device decodes such an agent as reject-all (O = 4) and
        # offer-nothing (C = 2), whichever of its two numbers was illegal, and counts it as bad
        aggregated=[dict(acceptor=13, offer=7, acc=[3, 2], off=[1, 2]),
                    dict(acceptor=24, offer=0, acc=[4, 4], off=[0, 0]),
                    dict(acceptor=25, offer=8, acc=[4, 4], off=[2, 2], bad=1),
                    dict(acceptor=0, offer=9, acc=[4, 4], off=[2, 2], bad=1)],
        fully=[dict(number=124, acc=[3, 2], off=[1, 2]), dict(number=224, acc=[4, 4], off=[2, 2]),
               dict(number=0, acc=[0, 0], off=[0, 0]), dict(number=225, acc=[4, 4], off=[2, 2], bad=1)])


def main():
    kats = [kat_wait_alternation(), kat_free_price_action0(), kat_auctioneer_ties(), kat_spawn_edge(),
            kat_self_offer_first_empty(), kat_mixed_chain(), kat_settlement_double_product(),
            kat_net_zero_offer_reward(), kat_noncommercial_price_reward(), kat_two_jobs_first_empty(),
            kat_hardcoded_agent_ties(), kat_liability_overflow(), kat_aggregated_chain_rewards(),
            kat_acception_quality()]
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats, f)
    with open(os.path.join(HERE, "kats_codec.json"), "w") as f:
        json.dump(codec_cases(), f)
    print("wrote %d scenarios + the codec cases" % len(kats))


if __name__ == "__main__":
    main()
