"""Synthetic action drivers shared by parity tests (test infrastructure)."""
import numpy as np


def random_actions(rng: np.random.Generator, obs_acc_counts, N, C, L, O, free, max_price, accept_bias=0.6):
    """Actions like a policy would emit them.

    obs_acc_counts[a][c] = number of real offers in acceptor (a, c)'s observation.
    Acceptors pick a real offer with probability accept_bias, else uniform in [0, O].
    Offer units pick a core action uniformly in [0, C]; with free prices the price
    follows FreePriceOfferPPO.selectAction (PPOmodules.py:312-332): -5 when the
    core chooser picked action 0, else uniform in [0, max_price].
    """
    acc = rng.integers(0, O + 1, size=(N, C))
    pick = rng.random((N, C)) < accept_bias
    for a in range(N):
        for c in range(C):
            n = int(obs_acc_counts[a][c])
            if pick[a, c] and n > 0:
                acc[a, c] = rng.integers(0, n)
    off = rng.integers(0, C + 1, size=(N, L))
    price = None
    if free:
        price = rng.integers(0, max_price + 1, size=(N, L))
        price[off == 0] = -5
    return acc.astype(np.int32), off.astype(np.int32), None if price is None else price.astype(np.int32)


def offer_counts_from_obs(acc_obs, O):
    """Number of non-pad (price, necT) pairs in each acceptor observation row."""
    pairs = np.asarray(acc_obs)[..., 3:3 + 2 * O].reshape(acc_obs.shape[:-1] + (O, 2))
    return (pairs[..., 1] != -2).sum(-1)
