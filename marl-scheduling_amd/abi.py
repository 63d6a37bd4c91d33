"""ctypes mirrors of include/marlsched.h (types only; no library is loaded here).

Kept separate from the loader so that test infrastructure (oracle/pyoracle.py)
can share the struct layouts without touching the product library.
"""
from __future__ import annotations

import ctypes as ct
import math

MAX_KINDS = 16
MAX_AGENTS = 64
MAX_CORES = 64
MAX_COLLECTION = 32
MAX_OFFERS = 126

OK = 0
EINVAL = 22
ENOMEM = 12
EHIP = 1001
EOVERFLOW = 75

FLAG_LIABILITY_OVERFLOW = 0x01
FLAG_BAD_ACTION = 0x02
FLAG_COLLECTION_FULL = 0x04
FLAG_SPAWN_EDGE = 0x08
FLAG_RNG_WINDOW = 0x10
FLAG_GUARD = 0x20

RNG_CPYTHON_MT19937 = 0


class MsConfig(ct.Structure):
    _fields_ = [
        ("n_agents", ct.c_int32),
        ("n_cores", ct.c_int32),
        ("collection_length", ct.c_int32),
        ("n_kinds", ct.c_int32),
        ("job_priority", ct.c_int32 * MAX_KINDS),
        ("job_length", ct.c_int32 * MAX_KINDS),
        ("acc_probability", ct.c_double * MAX_KINDS),
        ("n_fix_prices", ct.c_int32),
        ("fix_price", ct.c_int32 * MAX_KINDS),
        ("free_prices", ct.c_int32),
        ("commercial_reward", ct.c_int32),
        ("net_zero_offer_reward", ct.c_double),
        ("new_jobs_per_round", ct.c_int32),
        ("reward_multiplier", ct.c_int32),
        ("episode_length", ct.c_int32),
        ("liability_cap", ct.c_int32),
        ("rng_mode", ct.c_int32),
        ("reserved", ct.c_int32 * 7),
    ]


class MsShape(ct.Structure):
    _fields_ = [
        ("n_agents", ct.c_int32),
        ("n_cores", ct.c_int32),
        ("collection_length", ct.c_int32),
        ("max_offers", ct.c_int32),
        ("acc_obs_dim", ct.c_int32),
        ("acc_obs_stride", ct.c_int32),
        ("off_obs_dim", ct.c_int32),
        ("off_obs_stride", ct.c_int32),
        ("acc_actions", ct.c_int32),
        ("off_actions", ct.c_int32),
        ("price_actions", ct.c_int32),
        ("liability_cap", ct.c_int32),
        ("env_record_bytes", ct.c_int64),
    ]


class MsActions(ct.Structure):
    _fields_ = [
        ("acceptor", ct.c_void_p),
        ("offer_core", ct.c_void_p),
        ("offer_price", ct.c_void_p),
        ("auctioneer", ct.c_void_p),
    ]


class MsObsOut(ct.Structure):
    _fields_ = [("acceptor", ct.c_void_p), ("offer", ct.c_void_p), ("auctioneer", ct.c_void_p),
                ("core_rows", ct.c_void_p), ("core_owner", ct.c_void_p)]


class MsRewardOut(ct.Structure):
    _fields_ = [
        ("offer", ct.c_void_p),
        ("price", ct.c_void_p),
        ("acceptor", ct.c_void_p),
        ("auctioneer", ct.c_void_p),
        ("agent", ct.c_void_p),
        ("aggregated_offer", ct.c_void_p),
        ("aggregated_acceptor", ct.c_void_p),
    ]


class MsAcceptRec(ct.Structure):
    _fields_ = [
        ("valid", ct.c_int8),
        ("offerer", ct.c_int8),
        ("recipient", ct.c_int8),
        ("slot", ct.c_int8),
        ("price", ct.c_int8),
        ("nec_time", ct.c_int8),
        ("prio", ct.c_int8),
        ("kind", ct.c_int8),
        ("order", ct.c_int8),
        ("pad", ct.c_int8 * 3),
        ("round", ct.c_int32),
    ]


class MsTermRec(ct.Structure):
    _fields_ = [
        ("valid", ct.c_int8),
        ("owner", ct.c_int8),
        ("prio", ct.c_int8),
        ("init_len", ct.c_int8),
        ("dwell", ct.c_int32),
    ]


class MsEventOut(ct.Structure):
    _fields_ = [("accepted", ct.c_void_p), ("terminated", ct.c_void_p), ("launch_span", ct.c_void_p),
                ("metrics", ct.c_void_p), ("metrics_slots", ct.c_int32)]


class MsEnvMetrics(ct.Structure):
    """ms_env_metrics: one replica's episode accumulators (include/marlsched.h)."""
    _fields_ = [
        ("acceptor_reward", ct.c_int64),
        ("offer_reward", ct.c_int64),
        ("price_reward", ct.c_double),
        ("auctioneer_reward", ct.c_int64),
        ("termination_revenue", ct.c_int64),
        ("quality_sum", ct.c_double),
        ("quality_rounds", ct.c_int32),
        ("acception_amount", ct.c_int32),
        ("rounds", ct.c_int32),
        ("pad", ct.c_int32),
        ("price_sum", ct.c_int32 * MAX_KINDS),
        ("price_count", ct.c_int32 * MAX_KINDS),
        ("dwell_sum", ct.c_int32 * MAX_KINDS),
        ("dwell_count", ct.c_int32 * MAX_KINDS),
        ("agent_reward", ct.c_int64 * MAX_AGENTS),
    ]


METRICS_BYTES = ct.sizeof(MsEnvMetrics)


# numpy view of an [.., E] array of ms_env_metrics (field offsets from the ctypes struct)
def metrics_dtype():
    import numpy as np
    f = MsEnvMetrics
    names, formats, offsets = [], [], []
    for name, ctype in f._fields_:
        names.append(name)
        off = getattr(f, name).offset
        offsets.append(off)
        if name in ("price_sum", "price_count", "dwell_sum", "dwell_count"):
            formats.append((np.int32, MAX_KINDS))
        elif name == "agent_reward":
            formats.append((np.int64, MAX_AGENTS))
        else:
            formats.append({ct.c_int64: np.int64, ct.c_double: np.float64, ct.c_int32: np.int32}[ctype])
    return np.dtype(dict(names=names, formats=formats, offsets=offsets, itemsize=ct.sizeof(f)))


class MsStateHost(ct.Structure):
    _fields_ = [
        (name, ct.c_void_p)
        for name in (
            "round", "flags", "core_owner", "core_kind", "core_rem", "core_birth",
            "slot_kind", "slot_rem", "slot_wait", "slot_birth",
            "offer_core", "offer_recip", "offer_price", "liab_n", "liab", "mt", "mt_index",
        )
    ]


class MsMlpParams(ct.Structure):
    _fields_ = [
        ("w1", ct.c_void_p),
        ("b1", ct.c_void_p),
        ("w2", ct.c_void_p),
        ("b2", ct.c_void_p),
        ("w3", ct.c_void_p),
        ("b3", ct.c_void_p),
        ("in_dim", ct.c_int32),
        ("hidden", ct.c_int32),
        ("n_actions", ct.c_int32),
        ("n_groups", ct.c_int32),
        ("act_frag", ct.c_void_p),  # ms_act_prepare's block, or NULL
        ("row_base", ct.c_int64),   # the Philox row counter of row r is row_base + r (ABI 16)
    ]


class MsFusedAct(ct.Structure):  # ms_fused_act (ABI 16)
    _fields_ = [("offer", MsMlpParams), ("acceptor", MsMlpParams), ("common_row", ct.c_void_p), ("seed", ct.c_uint64),
                ("off_offset", ct.c_uint64), ("acc_offset", ct.c_uint64), ("offset_dev", ct.c_void_p),
                ("off_action", ct.c_void_p), ("off_logprob", ct.c_void_p), ("acc_action", ct.c_void_p),
                ("acc_logprob", ct.c_void_p)]


class MsRoundStrides(ct.Structure):  # ms_round_strides (ABI 16): bytes per round
    _fields_ = [(n, ct.c_int64) for n in ("acceptor_action", "offer_action", "core_rows", "core_owner", "offer_obs",
                                          "offer_reward", "acceptor_reward", "agent_reward", "auctioneer_reward",
                                          "next_off_action", "next_off_logprob", "next_acc_action",
                                          "next_acc_logprob")] + [("offset_step", ct.c_uint64)]


class MsFusedActFree(ct.Structure):  # ms_fused_act_free (ABI 18: own_action / own_logprob)
    _fields_ = [("core_chooser", MsMlpParams), ("price_chooser", MsMlpParams), ("acceptor", MsMlpParams),
                ("common_row", ct.c_void_p), ("price_table", ct.c_void_p), ("seed", ct.c_uint64),
                ("off_offset", ct.c_uint64), ("acc_offset", ct.c_uint64), ("offset_dev", ct.c_void_p)] + [
        (n, ct.c_void_p) for n in ("core_action", "core_logprob", "price_state", "price_action", "price_logprob",
                                   "env_price", "acc_action", "acc_logprob")] + [("defer_common", ct.c_int32),
                                                                                ("own_action", ct.c_void_p),
                                                                                ("own_logprob", ct.c_void_p)]


class MsRoundStridesFree(ct.Structure):  # ms_round_strides_free (ABI 18): bytes per round
    _fields_ = [(n, ct.c_int64) for n in ("acceptor_action", "offer_action", "core_rows", "core_owner", "offer_obs",
                                          "offer_reward", "price_reward", "acceptor_reward", "agent_reward",
                                          "auctioneer_reward", "next_core_action", "next_core_logprob",
                                          "next_price_state", "next_price_action", "next_price_logprob",
                                          "next_acc_action", "next_acc_logprob")] + [("offset_step", ct.c_uint64)] + [
        ("next_own_action", ct.c_int64), ("next_own_logprob", ct.c_int64)]


class MsQnetParams(ct.Structure):
    _fields_ = [("w1", ct.c_void_p), ("b1", ct.c_void_p), ("w2", ct.c_void_p), ("b2", ct.c_void_p),
                ("in_dim", ct.c_int32), ("hidden", ct.c_int32), ("n_actions", ct.c_int32), ("n_groups", ct.c_int32)]


class MsBdqnParams(ct.Structure):
    """ms_bdqn_params: one BranchingQNetwork, advantage heads stacked."""
    _fields_ = [("w1", ct.c_void_p), ("b1", ct.c_void_p), ("w2", ct.c_void_p), ("b2", ct.c_void_p),
                ("wv", ct.c_void_p), ("bv", ct.c_void_p), ("wa", ct.c_void_p), ("ba", ct.c_void_p),
                ("obs", ct.c_int32), ("ac_dim", ct.c_int32), ("n", ct.c_int32)]


class MsBdqnBatch(ct.Structure):
    """ms_bdqn_batch: one role's minibatch for ms_bdqn_update."""
    _fields_ = [("states", ct.c_void_p), ("next_states", ct.c_void_p), ("ld", ct.c_int32), ("actions", ct.c_void_p),
                ("actions_ld", ct.c_int32), ("rewards", ct.c_void_p), ("masks", ct.c_void_p), ("batch", ct.c_int32)]


class MsBdqnGrads(ct.Structure):
    _fields_ = [(k, ct.c_void_p) for k in ("w1", "b1", "w2", "b2", "wv", "bv", "wa", "ba", "loss")]


class MsDqnBatch(ct.Structure):
    _fields_ = [("states", ct.c_void_p), ("next_states", ct.c_void_p), ("actions", ct.c_void_p),
                ("rewards", ct.c_void_p), ("samples", ct.c_void_p), ("stride", ct.c_int32), ("n_units", ct.c_int32),
                ("units_per_group", ct.c_int32), ("capacity", ct.c_int32), ("batch", ct.c_int32),
                ("n_envs", ct.c_int64), ("gamma", ct.c_float)]


class MsQnetGrads(ct.Structure):
    _fields_ = [("w1", ct.c_void_p), ("b1", ct.c_void_p), ("w2", ct.c_void_p), ("b2", ct.c_void_p),
                ("loss", ct.c_void_p)]


class MsPpoBatch(ct.Structure):
    _fields_ = [
        ("states", ct.c_void_p),
        ("actions", ct.c_void_p),
        ("old_logprobs", ct.c_void_p),
        ("returns", ct.c_void_p),
        ("unit_of_group", ct.c_void_p),
        ("stride", ct.c_int32),
        ("T", ct.c_int32),
        ("U", ct.c_int32),
        ("E", ct.c_int64),
        ("common_row", ct.c_void_p),
        ("returns_ld", ct.c_int32),
        ("core_owner", ct.c_void_p),
        ("n_cores", ct.c_int32),
        ("row_keys", ct.c_int32),
        ("unit_stride", ct.c_int64),
    ]


class MsPriceTable(ct.Structure):
    _fields_ = [
        ("digit", ct.c_void_p),
        ("rows", ct.c_void_p),
        ("n_keys", ct.c_int32),
        ("table", ct.c_void_p),
    ]


class MsAdamTensor(ct.Structure):
    _fields_ = [
        ("param", ct.c_void_p),
        ("grad", ct.c_void_p),
        ("exp_avg", ct.c_void_p),
        ("exp_avg_sq", ct.c_void_p),
        ("numel", ct.c_int64),
        ("lr_group", ct.c_int32),
    ]


ADAM_MAX_TENSORS = 16


class MsWideBatch(ct.Structure):
    """ms_wide_batch: rollout rows of the aggregated nets (ms_wide_grad)."""
    _fields_ = [("states", ct.c_void_p), ("actions", ct.c_void_p), ("old_logprob", ct.c_void_p),
                ("returns", ct.c_void_p), ("stride", ct.c_int32), ("rows", ct.c_int64)]


class MsPpoGrads(ct.Structure):
    _fields_ = [(name, ct.c_void_p) for name in (
        "w1", "b1", "w2", "b2", "w3", "b3", "cw1", "cb1", "cw2", "cb2", "cw3", "cb3", "loss")]


ACCEPT_REC_BYTES = ct.sizeof(MsAcceptRec)
TERM_REC_BYTES = ct.sizeof(MsTermRec)
assert ACCEPT_REC_BYTES == 16 and TERM_REC_BYTES == 8


def accumulated_probabilities(probabilities):
    """world.accProbabilities (world.py:220-222): builtin sum, left to right."""
    return [sum(probabilities[: i + 1]) for i in range(len(probabilities))]


def make_config(
    n_agents,
    n_cores,
    collection_length,
    priorities,
    lengths,
    probabilities,
    fix_prices=None,
    free_prices=False,
    commercial=True,
    net_zero_offer_reward=0.5,
    new_jobs=1,
    reward_multiplier=1,
    episode_length=100,
    liability_cap=128,
) -> MsConfig:
    """Build an ms_config from World/Env parameters (world.py:211-246)."""
    if len(priorities) != len(lengths) or len(priorities) != len(probabilities):
        raise ValueError("priorities, lengths and probabilities must have equal length")
    if not 1 <= len(priorities) <= MAX_KINDS:
        raise ValueError("between 1 and %d job kinds" % MAX_KINDS)
    cfg = MsConfig()
    cfg.n_agents = n_agents
    cfg.n_cores = n_cores
    cfg.collection_length = collection_length
    cfg.n_kinds = len(priorities)
    for i, (p, l, a) in enumerate(zip(priorities, lengths, accumulated_probabilities(probabilities))):
        cfg.job_priority[i] = int(p)
        cfg.job_length[i] = int(l)
        cfg.acc_probability[i] = float(a)
    fix_prices = list(fix_prices or [])
    cfg.n_fix_prices = len(fix_prices)
    for i, p in enumerate(fix_prices[:MAX_KINDS]):
        cfg.fix_price[i] = int(p)
    cfg.free_prices = int(bool(free_prices))
    cfg.commercial_reward = int(bool(commercial))
    cfg.net_zero_offer_reward = float(net_zero_offer_reward)
    cfg.new_jobs_per_round = int(new_jobs)
    if int(reward_multiplier) != reward_multiplier:
        raise ValueError("rewardMultiplier must be an integer")
    cfg.reward_multiplier = int(reward_multiplier)
    cfg.episode_length = int(episode_length)
    cfg.liability_cap = int(liability_cap)
    cfg.rng_mode = RNG_CPYTHON_MT19937
    return cfg


def config_shape(cfg: MsConfig) -> dict:
    """Python mirror of ms_config_shape (for hosts without the library)."""
    O = cfg.n_agents * cfg.collection_length
    d_acc = 3 + 2 * O
    d_off = 2 * cfg.n_cores + 2
    return dict(
        N=cfg.n_agents,
        C=cfg.n_cores,
        L=cfg.collection_length,
        O=O,
        acc_obs_dim=d_acc,
        acc_obs_stride=(d_acc + 3) & ~3,
        off_obs_dim=d_off,
        off_obs_stride=(d_off + 3) & ~3,
        acc_actions=O + 1,
        off_actions=cfg.n_cores + 1,
        price_actions=max(cfg.job_priority[: cfg.n_kinds]) + 1,
        liability_cap=cfg.liability_cap or 128,
    )


# named configurations of BASELINE.json (README.md:49-61)
README_JOBS = dict(priorities=[3, 10], lengths=[6, 3], fix_prices=[2, 7], probabilities=[0.8, 0.2])
EXP4_JOBS = dict(priorities=[2, 4, 6, 8, 10, 12], lengths=[5] * 6, fix_prices=[1],
                 probabilities=[1 / 6] * 6)  # trainPPOExperiment4.py:48-51


def named_config(name: str) -> MsConfig:
    if name == "cfg1":  # trainPPO.py CPU reference: 2 agents, 2 cores, L=2, 2 job kinds, fixed prices
        return make_config(2, 2, 2, **README_JOBS)
    if name == "cfg2":  # 4 agents x 4 cores, fixed prices (globally shared PPO)
        return make_config(4, 4, 3, **README_JOBS)
    if name == "cfg3":  # 8 agents x 8 cores, free prices + commercial reward (locally shared PPO)
        return make_config(8, 8, 3, free_prices=True, commercial=True, **EXP4_JOBS)
    if name == "cfg4":  # 16 x 16, free prices
        return make_config(16, 16, 3, free_prices=True, commercial=True, **README_JOBS)
    if name == "cfg5":  # 32 x 32, free prices
        return make_config(32, 32, 3, free_prices=True, commercial=True, **README_JOBS)
    raise KeyError(name)


NAMED_ENVS = {"cfg1": 1, "cfg2": 4096, "cfg3": 16384, "cfg4": 65536, "cfg5": 65536}
assert math.isclose(sum(EXP4_JOBS["probabilities"]), 1.0)
