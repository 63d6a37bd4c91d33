"""Episode metrics of the training drivers from the env kernel's accumulators (ms_env_metrics).

The reference's drivers collect per episode (trainPPO.py:153-226, trainDQN.py:153-259):
accepted-offer prices per job kind, dwell times per job type, the accumulated unit rewards, the
auctioneer reward, the acception quality and amount (SchedulingEnvironment.py:174-192) and the
termination / trade revenues (Reward.py:193), and pickle them as ``argsDict``
(trainPPO.py:229-251) for Plot.py. Here ``ms_env_step`` adds every round into per-replica
accumulators on the device; this module turns one finished episode's accumulators into the
driver's per-episode values (per replica) and a list of episodes into an ``argsDict``.
"""
from __future__ import annotations

from fractions import Fraction
import statistics

import numpy as np

from . import abi


def view(raw) -> np.ndarray:
    """Host bytes [.., E, METRICS_BYTES] (uint8) -> structured array [.., E] of ms_env_metrics."""
    raw = np.ascontiguousarray(raw)
    return raw.view(abi.metrics_dtype()).reshape(raw.shape[:-1])


def episode_values(m: np.ndarray, cfg: abi.MsConfig, episode_length: int, n_agents: int, n_cores: int,
                   collection_length: int) -> list:
    """One finished episode, per replica: the values trainPPO.py:200-226 appends at ``done``.
    m: structured [E] (view()). Returns a list of E dicts."""
    K = cfg.n_kinds
    N, C, L, T = n_agents, n_cores, collection_length, episode_length
    prio = [cfg.job_priority[i] for i in range(K)]
    length = [cfg.job_length[i] for i in range(K)]
    # verweilzeiten are selected by (Prioritaet, Bedienzeit) (trainPPO.py:203): kinds sharing both
    # pool their terminations
    same = [[j for j in range(K) if prio[j] == prio[i] and length[j] == length[i]] for i in range(K)]
    out = []
    for r in m:
        d = {}
        # the accumulators are int64 torch tensors (float32 after "/ episodeLength"), except the core
        # chooser's under free prices, which `+=` of the float64 reward array turns into float64
        d["acceptorRew"] = float(np.float32(r["acceptor_reward"] / (T * N * C)))
        off = r["offer_reward"] / (T * N * L)
        d["coreChooserRew"] = float(off) if cfg.free_prices else float(np.float32(off))
        d["priceChooserRew"] = float(r["price_reward"] / (T * N * L))
        prices = []
        for i in range(K):
            n = int(r["price_count"][i])
            prices.append(float(Fraction(int(r["price_sum"][i]), n)) if n else None)
        d["prices"] = prices
        d["auctioneerRew"] = float(Fraction(int(r["auctioneer_reward"]), T))
        dwell = []
        for i in range(K):
            n = sum(int(r["dwell_count"][j]) for j in same[i])
            s = sum(int(r["dwell_sum"][j]) for j in same[i])
            dwell.append(float(Fraction(s, n * length[i])) if n else None)
        d["dwellTimes"] = dwell
        d["agentRew"] = r["agent_reward"][:N].astype(np.float64) / T
        qn = int(r["quality_rounds"])
        d["acceptionQuality"] = float(r["quality_sum"] / qn) if qn else None
        d["acceptionAmount"] = float(Fraction(int(r["acception_amount"]), T))
        d["terminationRevenues"] = float(r["termination_revenue"] / (T * N * C))
        d["tradeRevenues"] = 0.0  # Reward.py:110,179: the trade revenue update is commented out
        d["rounds"] = int(r["rounds"])
        out.append(d)
    return out


LIST_KEYS = ("acceptorRew", "coreChooserRew", "priceChooserRew", "prices", "auctioneerRew", "dwellTimes",
             "agentRew", "acceptionQuality", "acceptionAmount", "terminationRevenues", "tradeRevenues")


def _mean_opt(vals):
    vals = [v for v in vals if v is not None]
    return float(np.mean(vals)) if vals else None


def reduce_replicas(per_replica: list) -> dict:
    """One episode's values averaged over replicas (None where no replica had a value)."""
    out = {}
    for k in LIST_KEYS:
        vs = [d[k] for d in per_replica]
        if k in ("prices", "dwellTimes"):
            out[k] = [_mean_opt([v[i] for v in vs]) for i in range(len(vs[0]))]
        elif k == "agentRew":
            out[k] = np.mean(np.stack(vs), axis=0)
        else:
            out[k] = _mean_opt(vs)
    return out


def args_dict(episodes: list, cfg: abi.MsConfig, params: dict | None = None, replica="mean",
              plot_path: str = "") -> dict:
    """argsDict of trainPPO.py:229-243 from a list of episodes (each a list of per-replica dicts
    from episode_values). replica = "mean" averages over replicas, an int picks one replica."""
    eps = [reduce_replicas(ep) if replica == "mean" else ep[int(replica)] for ep in episodes]
    K = cfg.n_kinds
    d = {"plotPath": plot_path}
    names = dict(acceptorRew="acceptorRew", coreChooserRew="coreChooserRew", priceChooserRew="priceChooserRew",
                 prices="prices", auctioneerRew="auctioneerRew", dwellTimes="dwellTimes", agentRew="agentRew",
                 acceptionQuality="acceptionQuality", acceptionAmount="acceptionAmount",
                 terminationRevenues="terminationRevenues", tradeRevenues="tradeRevenues")
    for k in LIST_KEYS:
        d[names[k]] = [e[k] for e in eps]
    # meanJobFraction = statistics.mean of Fraction(prio, len) over the job kinds (trainPPO.py:49-50)
    d["meanJob"] = statistics.mean([Fraction(cfg.job_priority[i], cfg.job_length[i]) for i in range(K)])
    d["params"] = dict(params or {})
    return d


def save_args_dict(d: dict, file_name: str = "data{}.pkl", directory: str = ".") -> str:
    """Pickle an argsDict the way trainPPO.py:245-251 does: the first ``file_name.format(i)``
    (i = 0, 1, ...) that does not exist yet, so the reference's Plot.py reads it. Returns the path."""
    import os
    import pickle

    i = 0
    while os.path.isfile(os.path.join(directory, file_name.format(i))):
        i += 1
    path = os.path.join(directory, file_name.format(i))
    with open(path, "wb") as f:
        pickle.dump(d, f)
    return path
