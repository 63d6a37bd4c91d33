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


def main():
    kats = [kat_wait_alternation(), kat_free_price_action0(), kat_auctioneer_ties(), kat_spawn_edge(),
            kat_self_offer_first_empty(), kat_mixed_chain(), kat_settlement_double_product()]
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats, f)
    print("wrote %d scenarios" % len(kats))


if __name__ == "__main__":
    main()
