"""Aggregated agents on the CPU: the action codec restatement (Agent.py:644-666) and the
aggregated observation / reward restatement (oracle/pyref.py) on hand-checked cases."""
import itertools

import pytest

from oracle import pyref


@pytest.mark.parametrize("base,dim", [(5, 2), (3, 2), (13, 4), (2, 5)])
def test_number_to_nd_action_is_little_endian_digits(base, dim):
    for number in range(base ** dim):
        digits = pyref.number_to_nd_action(number, base, dim)
        assert digits == [(number // base ** i) % base for i in range(dim)]
    with pytest.raises(ValueError):
        pyref.number_to_nd_action(base ** dim, base, dim)
    with pytest.raises(ValueError):
        pyref.number_to_nd_action(-1, base, dim)


def test_aggregated_observations_and_rewards_kat():
    cfg = pyref.Config(n_agents=2, n_cores=2, collection_length=2, priorities=[3, 10], lengths=[6, 3],
                       probabilities=[0.8, 0.2], fix_prices=[2, 7])
    w = pyref.PyWorld(cfg, 0)
    acc, off, fully = w.aggregated_obs()
    O = 4
    assert len(acc[0]) == 2 * (3 + 2 * O) and len(off[0]) == 2 * 2 + 2 * 2
    assert fully[1] == off[1] + acc[1]
    # round 0: empty world -> acceptor rows [0,-1,-1, -2...] per core, offer rows all -1
    assert acc[0] == ([0, -1, -1] + [-2] * (2 * O)) * 2 and off[0] == [-1] * 8
    # offer every slot to core 1 every round, accept the first offer everywhere: once jobs exist,
    # executions and terminations happen, and the aggregated rewards follow Reward.py:92-143
    saw_term = False
    for _ in range(40):
        w.step([[0, 0], [0, 0]], [[0, 0], [0, 0]])
        agg_off, agg_acc = w.last_aggregated
        assert agg_off[:, 0].tolist() == [sum(o.prio1 for o in w.accepted if o.offerer == a + 1) for a in range(2)]
        saw_term |= bool(w.term)
        a, o, f = w.aggregated_obs()
        for ag in range(2):
            assert o[ag][:4] == [v for c in range(2) for v in (w.core_job[c].prio, w.core_job[c].rem)]
            assert list(itertools.chain(*[w.acceptor_obs(ag, c) for c in range(2)])) == a[ag]
    assert saw_term
