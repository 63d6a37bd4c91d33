"""PPO for groups of tiny actor-critics (PPOmodules.py, batched over units and replicas).

The reference keeps one ``ActorCritic`` per unit (PPOmodules.py:25-72) and
updates each with its own ``PPO.update`` (PPOmodules.py:127-174). Here the
nets of one unit type are stacked into groups ``[G, ...]``:

* divided agents   — one group per unit (``AcceptorPPO``/``OfferPPO``/``FreePriceOfferPPO``),
* locally shared   — one group per agent (``LocallySharedPPO``, PPOmodules.py:490-597),
* globally shared  — one group (``GloballySharedPPO``, PPOmodules.py:335-449).

Action selection runs in the fused HIP kernel (``ms_policy_act``). The update's
gradient comes from the fused HIP kernel (``ms_ppo_grad``: forward, loss and
backward of every group in one launch) and the HIP Adam step (``ms_adam_step``)
applies it on two parameter groups (actor / critic learning rates,
PPOmodules.py:100-105); ``PPOGroup.update`` keeps a torch-autograd twin with
``torch.optim.Adam`` as the numerical reference. All groups step in lockstep,
which equals independent per-net optimizers because Adam is elementwise. With E replicas a sub-unit's batch holds its
E*T transitions; returns are normalised per replica over T so that E = 1 is
exactly the reference.
"""
from __future__ import annotations

import contextlib
import ctypes as ct

import torch
import torch.nn as nn
from torch.distributions import Categorical

from . import abi
from ._lib import check, lib, ptr, stream_ptr

MS_EINVAL = 22  # include/marlsched.h

HIDDEN = 16  # numberOfNeurons of every divided / shared net (PPOmodules.py:241,259,276,456,475,604,623)


def reference_actor_critic_params(in_dim: int, n_actions: int, hidden: int = HIDDEN):
    """One ActorCritic initialised exactly like the reference constructor:
    actor Linear x3 then critic Linear x3 with nn.Linear's default init on the
    current torch CPU generator (PPOmodules.py:32-48). Returns a flat dict."""
    a1, a2, a3 = nn.Linear(in_dim, hidden), nn.Linear(hidden, hidden), nn.Linear(hidden, n_actions)
    c1, c2, c3 = nn.Linear(in_dim, hidden), nn.Linear(hidden, hidden), nn.Linear(hidden, 1)
    return dict(w1=a1.weight, b1=a1.bias, w2=a2.weight, b2=a2.bias, w3=a3.weight, b3=a3.bias,
                cw1=c1.weight, cb1=c1.bias, cw2=c2.weight, cb2=c2.bias, cw3=c3.weight, cb3=c3.bias)


def reference_nets(order, dims):
    """ActorCritic parameter dicts in the reference's construction order: each PPO object makes
    policy then policy_old (PPOmodules.py:99,107) on torch's CPU generator. order: list of unit-type
    names in construction order; dims: name -> (in_dim, n_actions). Returns name -> [dict, ...]."""
    nets = {k: [] for k in dims}
    for name in order:
        D, A = dims[name]
        nets[name].append(reference_actor_critic_params(D, A))
        reference_actor_critic_params(D, A)  # policy_old: same init stream, then overwritten
    return nets


def reference_init_order(arch: str, N: int, C: int, L: int, free: bool):
    """Unit types in the order the reference's agents construct their PPO objects:
    divided — per agent C acceptors then L offer units (Agent.py:495-502; free prices: coreChooser,
    priceChooser per slot, Agent.py:589-596, PPOmodules.py:277-306); locally shared — per agent the
    shared acceptor then the shared offer unit(s) (Agent.py:669-680); globally shared — one acceptor
    then the offer unit(s) (SchedulingEnvironment.py:269-275)."""
    off_units = ["off", "price"] if free else ["off"]
    if arch == "divided":
        return [u for _ in range(N) for u in ["acc"] * C + off_units * L]
    if arch == "local":
        return [u for _ in range(N) for u in ["acc"] + off_units]
    return ["acc"] + off_units


ACTOR_KEYS = ("w1", "b1", "w2", "b2", "w3", "b3")
CRITIC_KEYS = ("cw1", "cb1", "cw2", "cb2", "cw3", "cb3")


class GroupedActorCritic(nn.Module):
    """G ActorCritic nets of identical shape, parameters stacked along dim 0."""

    def __init__(self, n_groups: int, in_dim: int, n_actions: int, hidden: int = HIDDEN, init: bool = True):
        super().__init__()
        self.G, self.D, self.A, self.H = n_groups, in_dim, n_actions, hidden
        if not init:
            shapes = dict(w1=(hidden, in_dim), b1=(hidden,), w2=(hidden, hidden), b2=(hidden,), w3=(n_actions, hidden),
                          b3=(n_actions,), cw1=(hidden, in_dim), cb1=(hidden,), cw2=(hidden, hidden), cb2=(hidden,),
                          cw3=(1, hidden), cb3=(1,))
            for k in ACTOR_KEYS + CRITIC_KEYS:
                self.register_parameter(k, nn.Parameter(torch.zeros((n_groups,) + shapes[k])))
            return
        nets = []
        for _ in range(n_groups):
            # the reference builds policy then policy_old (PPOmodules.py:99,107): both draw
            # from torch's generator, so construct both to keep the same init stream.
            p = reference_actor_critic_params(in_dim, n_actions, hidden)
            reference_actor_critic_params(in_dim, n_actions, hidden)
            nets.append(p)
        for k in ACTOR_KEYS + CRITIC_KEYS:
            self.register_parameter(k, nn.Parameter(torch.stack([n[k].detach() for n in nets]).contiguous()))

    @classmethod
    def from_params(cls, nets: list, in_dim: int, n_actions: int, hidden: int = HIDDEN):
        """Stack per-net parameter dicts (reference_actor_critic_params) into one grouped module,
        for callers that build the nets of several unit types in the reference's interleaved order."""
        m = cls(len(nets), in_dim, n_actions, hidden, init=False)
        with torch.no_grad():
            for k in ACTOR_KEYS + CRITIC_KEYS:
                getattr(m, k).copy_(torch.stack([n[k].detach() for n in nets]))
        return m

    def actor_parameters(self):
        return [getattr(self, k) for k in ACTOR_KEYS]

    def critic_parameters(self):
        return [getattr(self, k) for k in CRITIC_KEYS]

    @staticmethod
    def _mlp(x, w1, b1, w2, b2, w3, b3):
        h = torch.tanh(torch.baddbmm(b1.unsqueeze(1), x, w1.transpose(1, 2)))
        h = torch.tanh(torch.baddbmm(b2.unsqueeze(1), h, w2.transpose(1, 2)))
        return torch.baddbmm(b3.unsqueeze(1), h, w3.transpose(1, 2))

    def actor_probs(self, x):
        """x [G, R, D] float -> action probabilities [G, R, A] (nn.Softmax(dim=-1))."""
        return torch.softmax(self._mlp(x, self.w1, self.b1, self.w2, self.b2, self.w3, self.b3), dim=-1)

    def critic(self, x):
        return self._mlp(x, self.cw1, self.cb1, self.cw2, self.cb2, self.cw3, self.cb3).squeeze(-1)

    def evaluate(self, x, actions):
        """ActorCritic.evaluate (PPOmodules.py:65-72) batched over groups."""
        dist = Categorical(self.actor_probs(x))
        return dist.log_prob(actions), self.critic(x), dist.entropy()

    def mlp_params(self, frag: "ActFrag | None" = None, row_base: int = 0) -> abi.MsMlpParams:
        """The actor's ms_mlp_params; frag: an ActFrag built for the current weights (acting only);
        row_base: the Philox row counter of the call's first row (acting only)."""
        for k in ACTOR_KEYS:
            t = getattr(self, k)
            assert t.is_cuda and t.is_contiguous() and t.dtype == torch.float32
        return abi.MsMlpParams(ptr(self.w1), ptr(self.b1), ptr(self.w2), ptr(self.b2), ptr(self.w3), ptr(self.b3),
                               self.D, self.H, self.A, self.G, ptr(frag.buf) if frag is not None else None,
                               int(row_base))

    def critic_mlp_params(self) -> abi.MsMlpParams:
        return abi.MsMlpParams(ptr(self.cw1), ptr(self.cb1), ptr(self.cw2), ptr(self.cb2), ptr(self.cw3),
                               ptr(self.cb3), self.D, self.H, 1, self.G)

    @torch.no_grad()
    def act(self, obs_i8, n_units: int, seed: int, offset: int, uniforms=None, action=None, logprob=None, stream=None,
            offset_dev=None, common_row=None, frag: "ActFrag | None" = None, replica_base: int = 0):
        """ActorCritic.act (PPOmodules.py:53-63) for obs [E, n_units, stride] int8 on the HIP kernel.
        Unit u uses group u // (n_units // G). Returns (action int8 [E, U], logprob f32 [E, U]).
        common_row (int8 [stride] on the device, optional): rows equal to it share one forward pass
        (``ms_policy_act_common``; same outputs). replica_base: the global index of obs's first replica
        (its Philox rows start at replica_base * n_units: a shard draws what the whole set would)."""
        E, U, stride = obs_i8.shape
        assert U == n_units and U % self.G == 0 and obs_i8.dtype == torch.int8 and obs_i8.is_contiguous()
        dev = obs_i8.device
        if action is None:
            action = torch.empty((E, U), dtype=torch.int8, device=dev)
        if logprob is None:
            logprob = torch.empty((E, U), dtype=torch.float32, device=dev)
        p = self.mlp_params(frag, replica_base * U)
        if common_row is not None:
            assert common_row.dtype == torch.int8 and common_row.numel() == stride and common_row.device == dev
            check(lib.ms_policy_act_common(ct.byref(p), ptr(obs_i8), stride, E, U, U // self.G, ptr(common_row),
                                           ct.c_uint64(seed), ct.c_uint64(offset), ptr(offset_dev), ptr(uniforms),
                                           ptr(action), ptr(logprob), stream_ptr(stream)))
            return action, logprob
        check(lib.ms_policy_act(ct.byref(p), ptr(obs_i8), stride, E, U, U // self.G, ct.c_uint64(seed),
                                ct.c_uint64(offset), ptr(offset_dev), ptr(uniforms), ptr(action), ptr(logprob),
                                stream_ptr(stream)))
        return action, logprob

    @torch.no_grad()
    def act_compact(self, core_rows, core_owner, n_units: int, seed: int, offset: int, common_row, uniforms=None,
                    action=None, logprob=None, stream=None, offset_dev=None, frag: "ActFrag | None" = None,
                    replica_base: int = 0):
        """``act`` with common_row on compact acceptor observations (ms_policy_act_compact):
        core_rows [E, C, stride], core_owner [E, C] int8; unit u = a*C + c acts on core row c when
        core_owner == a + 1, else on common_row. Same outputs as ``act`` on the regenerated rows."""
        E, C, stride = core_rows.shape
        assert core_rows.dtype == torch.int8 and core_rows.is_contiguous() and core_owner.is_contiguous()
        assert core_owner.shape == (E, C) and n_units % C == 0 and n_units % self.G == 0
        dev = core_rows.device
        if action is None:
            action = torch.empty((E, n_units), dtype=torch.int8, device=dev)
        if logprob is None:
            logprob = torch.empty((E, n_units), dtype=torch.float32, device=dev)
        p = self.mlp_params(frag, replica_base * n_units)
        check(lib.ms_policy_act_compact(ct.byref(p), ptr(core_rows), ptr(core_owner), stride, E, n_units,
                                        n_units // self.G, C, ptr(common_row), ct.c_uint64(seed), ct.c_uint64(offset),
                                        ptr(offset_dev), ptr(uniforms), ptr(action), ptr(logprob), stream_ptr(stream)))
        return action, logprob


class PriceTable:
    """The price chooser's sampling table (ms_price_table): the inputs the env can hand it are
    [prio, rem] of a core and of the offer slot (Agent.py:271-300) or the dummy [-5, -5, -5, -5]
    (PPOmodules.py:327); every row with prio in {-5, -1, 0 .. max priority} and rem in
    {-5, -1, 0 .. max length} is a key, and ``build`` tabulates the net's sampling entries for the
    current weights (a row outside the table makes its tile compute the net, as without one)."""

    def __init__(self, cfg, price: "GroupedActorCritic"):
        kinds = int(cfg.n_kinds)
        prios = [-5, -1] + list(range(0, max(int(p) for p in cfg.job_priority[:kinds]) + 1))
        rems = [-5, -1] + list(range(0, max(int(x) for x in cfg.job_length[:kinds]) + 1))
        sets = [prios, rems, prios, rems]
        dev = price.w1.device
        digit = torch.full((4, 256), -1, dtype=torch.int16)
        stride = 1
        for pos, vals in enumerate(sets):
            for i, v in enumerate(vals):
                digit[pos, v + 128] = i * stride
            stride *= len(vals)
        self.n_keys = stride
        grids = torch.meshgrid(*[torch.tensor(v, dtype=torch.int8) for v in reversed(sets)], indexing="ij")
        rows = torch.stack([g.reshape(-1) for g in reversed(grids)], 1)  # key = sum of digit offsets
        self.digit = digit.to(dev)
        self.rows = rows.contiguous().to(dev)
        tw = 32 * ((price.A + 15) // 16) + 4
        self.table = torch.zeros((price.G, self.n_keys, tw), dtype=torch.float32, device=dev)
        self.struct = abi.MsPriceTable(ptr(self.digit), ptr(self.rows), self.n_keys, ptr(self.table))

    def build(self, price: "GroupedActorCritic", stream=None):
        p = price.mlp_params()
        check(lib.ms_price_table_build(ct.byref(p), ct.byref(self.struct), stream_ptr(stream)))


class ActFrag:
    """ms_act_prepare's block for one net acting on rows of ``stride`` bytes (with ``common_row``, also
    the common row's sampling table): each acting lane's weight fragments, made once from the current
    weights instead of by every acting wave of every round (the acting net, policy_old, changes only
    at updates: PPOmodules.py:171). ``build`` it after every weight change; acting with it is
    bit-identical to acting without."""

    def __init__(self, net: "GroupedActorCritic", stride: int, common_row=None):
        self.stride, self.common_row = int(stride), common_row
        p = net.mlp_params()
        n = lib.ms_act_frag_bytes(ct.byref(p), self.stride)
        assert n > 0, "no act fragments for this net shape"
        self.buf = torch.zeros(n, dtype=torch.uint8, device=net.w1.device)

    def build(self, net: "GroupedActorCritic", stream=None):
        p = net.mlp_params()
        check(lib.ms_act_prepare(ct.byref(p), ptr(self.common_row), self.stride, ptr(self.buf), stream_ptr(stream)))


@torch.no_grad()
def act_round_free(core: GroupedActorCritic, price: GroupedActorCritic, off_obs, acc: GroupedActorCritic, core_rows,
                   core_owner, common_row, n_cores: int, seed: int, off_offset: int, acc_offset: int, out: dict,
                   acc_action, acc_logprob, offset_dev=None, stream=None, price_table: PriceTable | None = None,
                   price_unit_stride: int = 0, core_frag: "ActFrag | None" = None, acc_frag: "ActFrag | None" = None,
                   replica_base: int = 0):
    """``offer_act_free`` + ``act_compact`` of one free-price round in one launch (ms_act_round_free):
    getActionForAllAgents (SchedulingEnvironment.py:150-172); outputs identical to the two calls. price None:
    a fixed-price round, ``core.act`` of the offer units + ``act_compact`` (out: core_action / core_logprob).
    price_table: the price chooser samples from it (built for the current weights).
    price_unit_stride: see ``offer_act_free``. core_frag / acc_frag: ActFrag blocks of the core chooser and
    the acceptor net for their current weights (bit-identical; the acting waves then skip deriving them)."""
    E, U_off, off_stride = off_obs.shape
    _, C, acc_stride = core_rows.shape
    U_acc = acc_action.shape[1]
    assert off_obs.is_contiguous() and core_rows.is_contiguous() and core_owner.is_contiguous()
    pc = core.mlp_params(core_frag, replica_base * U_off)
    pa = acc.mlp_params(acc_frag, replica_base * U_acc)
    if price is None:  # a fixed-price round: out holds core_action / core_logprob only
        assert price_table is None and price_unit_stride == 0
        for k in ("core_action", "core_logprob"):
            assert out[k].is_contiguous() and out[k].shape[:2] == (E, U_off), k
        pp, prices = None, (None, None, None, None)
    else:
        _check_price_out(out, E, U_off, price_unit_stride)
        pp = ct.byref(price.mlp_params())
        prices = (out["price_state"], out["price_action"], out["price_logprob"], out["env_price"])
    check(lib.ms_act_round_free(ct.byref(pc), pp, ptr(off_obs), off_stride, U_off, U_off // core.G,
                                ct.byref(pa), ptr(core_rows), ptr(core_owner), acc_stride, U_acc, U_acc // acc.G,
                                n_cores, ptr(common_row), E, ct.c_uint64(seed), ct.c_uint64(off_offset),
                                ct.c_uint64(acc_offset), ptr(offset_dev), ptr(out["core_action"]),
                                ptr(out["core_logprob"]), *[ptr(x) for x in prices], ptr(acc_action), ptr(acc_logprob),
                                ct.byref(price_table.struct) if price_table is not None else None,
                                int(price_unit_stride), stream_ptr(stream)))


def _check_price_out(out, E: int, U: int, pus: int):
    """The price chooser's outputs: [E, U(, 4)] contiguous (pus = 0), or unit-major [U, E(, 4)] views
    whose unit stride (in rows) is pus."""
    for k in ("price_state", "price_action", "price_logprob"):
        x = out[k]
        if pus == 0:
            assert x.is_contiguous() and x.shape[:2] == (E, U), k
        else:
            assert x.shape[:2] == (U, E) and x.stride(1) == x[0, 0].numel() and pus >= E, k
            assert x.stride(0) == pus * x[0, 0].numel(), k


def regen_acceptor_rows(core_rows, core_owner, common_row, n_agents: int):
    """The [..., N*C, stride] acceptor rows of compact observations (core_rows [..., C, stride],
    core_owner [..., C]): row (a, c) = core_rows[c] if core_owner[c] == a + 1 else common_row
    (Agent.py:167-212). Torch ops, for the reference update path and tests."""
    C = core_rows.shape[-2]
    agents = torch.arange(1, n_agents + 1, device=core_rows.device, dtype=core_owner.dtype)
    own = core_owner.unsqueeze(-2) == agents.view(n_agents, 1)                  # [..., N, C]
    rows = torch.where(own.unsqueeze(-1), core_rows.unsqueeze(-3), common_row)  # [..., N, C, stride]
    return rows.reshape(rows.shape[:-3] + (n_agents * C, rows.shape[-1]))


@torch.no_grad()
def offer_act_free(core: GroupedActorCritic, price: GroupedActorCritic, obs_i8, n_cores: int, seed: int, offset: int,
                   out: dict, uniforms=None, offset_dev=None, stream=None, price_unit_stride: int = 0,
                   core_frag: "ActFrag | None" = None, replica_base: int = 0):
    """FreePriceOfferPPO.selectAction (PPOmodules.py:312-332) for obs [E, U, stride] int8 in one launch.
    out: core_action/price_action/env_price int8 [E, U], core_logprob/price_logprob f32 [E, U],
    price_state int8 [E, U, 4]. price_unit_stride > 0: price_state / price_action / price_logprob are
    unit-major views [U, E(, 4)] of a ring whose units lie price_unit_stride rows apart."""
    E, U, stride = obs_i8.shape
    assert obs_i8.dtype == torch.int8 and obs_i8.is_contiguous() and U % core.G == 0
    _check_price_out(out, E, U, price_unit_stride)
    pc, pp = core.mlp_params(core_frag, replica_base * U), price.mlp_params()
    check(lib.ms_offer_act_free(ct.byref(pc), ct.byref(pp), ptr(obs_i8), stride, E, U, U // core.G, n_cores,
                                ct.c_uint64(seed), ct.c_uint64(offset), ptr(offset_dev), ptr(uniforms),
                                ptr(out["core_action"]), ptr(out["core_logprob"]), ptr(out["price_state"]),
                                ptr(out["price_action"]), ptr(out["price_logprob"]), ptr(out["env_price"]),
                                int(price_unit_stride), stream_ptr(stream)))
    return out


def discounted_returns(rewards_tm: torch.Tensor, gamma: float, stream=None) -> torch.Tensor:
    """PPO.update's return estimate (PPOmodules.py:128-137) on the HIP kernel.
    rewards_tm [T, M] f32 (time-major, M independent sequences) -> [M, T] f32 normalised per sequence."""
    rewards_tm = rewards_tm.contiguous().float()
    T, M = rewards_tm.shape
    out = torch.empty((M, T), dtype=torch.float32, device=rewards_tm.device)
    check(lib.ms_discounted_returns(ptr(rewards_tm), T, M, M, ct.c_double(gamma), ptr(out), stream_ptr(stream)))
    return out


def unit_returns(rewards_teu: torch.Tensor, unit_of_group: torch.Tensor, gamma: float, stream=None) -> torch.Tensor:
    """PPO.update's return estimate (PPOmodules.py:128-137) for the unit each group trains on, read
    straight from the rollout rewards [T, E, U] (f32 or int32). unit_of_group [G] int32 on the device.
    Returns [T, E, G] f32 normalised per (replica, group) sequence (the ms_ppo_batch layout)."""
    assert rewards_teu.dim() == 3 and rewards_teu.is_contiguous()
    assert rewards_teu.dtype in (torch.float32, torch.int32) and unit_of_group.dtype == torch.int32
    T, E, U = rewards_teu.shape
    G = unit_of_group.numel()
    out = torch.empty((T, E, G), dtype=torch.float32, device=rewards_teu.device)
    check(lib.ms_unit_returns(ptr(rewards_teu), int(rewards_teu.dtype == torch.int32), T, E, U, ptr(unit_of_group),
                              G, ct.c_double(gamma), ptr(out), stream_ptr(stream)))
    return out


def combine_losses(terms):
    """PPO.update's loss (PPOmodules.py:157-159) per group from ms_ppo_grad's [..., 3] terms (mean -min(surr),
    mean (V - G)^2, mean entropy): -min + 0.5 * mse - 0.01 * entropy, the same f32 operations for one epoch's
    [G][3] or several epochs' stacked [n][G][3]."""
    return terms[..., 0] + 0.5 * terms[..., 1] - 0.01 * terms[..., 2]


class HipAdam:
    """torch.optim.Adam (defaults betas (0.9, 0.999), eps 1e-8, no weight decay) over the
    parameters of one PPOGroup as one ``ms_adam_step`` launch per step: tensor i of
    ``param_groups[k]["params"]`` uses ``param_groups[k]["lr"]`` like torch's param groups
    (PPOmodules.py:100-105). The state (exp_avg, exp_avg_sq, step) mirrors torch's."""

    def __init__(self, param_groups, betas=(0.9, 0.999), eps=1e-8):
        self.param_groups = [dict(params=list(g["params"]), lr=float(g["lr"])) for g in param_groups]
        self.betas, self.eps = betas, eps
        self.step_count = 0
        self.state = {}
        # the step count on the device as well: each step advances it with a device op and the Adam
        # kernel reads it, so a captured HIP graph (Trainer's update) replays with the current count
        dev = self.param_groups[0]["params"][0].device
        self.step_dev = torch.zeros((), dtype=torch.int64, device=dev)
        for g in self.param_groups:
            for p in g["params"]:
                assert p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                self.state[p] = dict(exp_avg=torch.zeros_like(p), exp_avg_sq=torch.zeros_like(p))
        n = sum(len(g["params"]) for g in self.param_groups)
        assert n <= abi.ADAM_MAX_TENSORS and len(self.param_groups) <= 4

    def zero_grad(self):
        for g in self.param_groups:
            for p in g["params"]:
                p.grad = None

    @torch.no_grad()
    def step(self, stream=None):
        self.step_count += 1
        if stream is None:
            self.step_dev.add_(1)
        else:
            with torch.cuda.stream(stream):
                self.step_dev.add_(1)
        ts = []
        for k, g in enumerate(self.param_groups):
            for p in g["params"]:
                if p.grad is None:  # torch skips parameters without a gradient
                    continue
                st = self.state[p]
                ts.append(abi.MsAdamTensor(ptr(p), ptr(p.grad), ptr(st["exp_avg"]), ptr(st["exp_avg_sq"]), p.numel(), k))
        if not ts:
            return
        arr = (abi.MsAdamTensor * len(ts))(*ts)
        lrs = (ct.c_double * len(self.param_groups))(*[g["lr"] for g in self.param_groups])
        check(lib.ms_adam_step_dev(arr, len(ts), lrs, len(self.param_groups), ptr(self.step_dev), self.betas[0],
                                   self.betas[1], self.eps, stream_ptr(stream)))


def _on_stream(stream):
    """torch.cuda.stream(stream), or no change for stream None (the current stream)."""
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


class PPOGroup:
    """Policy / policy_old pair + Adam for one unit type (PPOmodules.py:75-174). The torch-autograd
    ``update`` steps torch.optim.Adam; ``update_fused`` steps the HIP Adam (HipAdam)."""

    def __init__(self, n_groups, in_dim, n_actions, lr_actor, lr_critic, gamma, eps_clip, k_epochs, device,
                 allreduce=None, init_nets=None, hidden: int = HIDDEN):
        if init_nets is not None:  # per-group parameter dicts built by the caller, in reference order
            assert len(init_nets) == n_groups
            self.policy = GroupedActorCritic.from_params(init_nets, in_dim, n_actions, hidden).to(device)
        else:
            self.policy = GroupedActorCritic(n_groups, in_dim, n_actions, hidden).to(device)
        self.policy_old = GroupedActorCritic(n_groups, in_dim, n_actions, hidden, init=False).to(device)
        self.policy_old.requires_grad_(False)
        self.sync_old()
        self.param_groups = [
            {"params": self.policy.actor_parameters(), "lr": lr_actor},
            {"params": self.policy.critic_parameters(), "lr": lr_critic},
        ]
        self._torch_opt = self._hip_opt = None
        self.gamma, self.eps_clip, self.K = gamma, eps_clip, k_epochs
        self.allreduce = allreduce
        self.last_losses = []

    @property
    def optimizer(self):
        """torch.optim.Adam of the torch-autograd path (created on first use)."""
        if self._torch_opt is None:
            self._torch_opt = torch.optim.Adam([dict(g) for g in self.param_groups])
        return self._torch_opt

    @property
    def hip_optimizer(self):
        """HipAdam of the fused path (created on first use)."""
        if self._hip_opt is None:
            self._hip_opt = HipAdam(self.param_groups)
        return self._hip_opt

    @torch.no_grad()
    def wide_act(self, obs_i8, uniforms=None, action=None, logprob=None, generator=None, stream=None):
        """PPO.selectAction + ActorCritic.act (PPOmodules.py:53-63, 114-125) of the aggregated agents'
        nets (32 / 64 hidden units, (O+1)^C-sized action spaces; ms_wide_act): row (e, g) of obs
        [E, G, stride] int8 through group g's policy_old, the action drawn by inverse CDF at
        uniforms [E, G] (default: torch.rand on the device). Returns (action int32 [E, G],
        log-prob f32 [E, G]), written into ``action`` / ``logprob`` when given."""
        E, G, stride = obs_i8.shape
        pol = self.policy_old
        assert G == pol.G and obs_i8.dtype == torch.int8 and obs_i8.is_contiguous() and stride >= pol.D
        dev = obs_i8.device
        if uniforms is None:
            uniforms = torch.rand((E, G), device=dev, generator=generator)
        assert uniforms.shape == (E, G) and uniforms.dtype == torch.float32 and uniforms.is_contiguous()
        if action is None:
            action = torch.empty((E, G), dtype=torch.int32, device=dev)
        if logprob is None:
            logprob = torch.empty((E, G), dtype=torch.float32, device=dev)
        assert action.dtype == torch.int32 and action.is_contiguous() and action.shape == (E, G)
        assert logprob.dtype == torch.float32 and logprob.is_contiguous() and logprob.shape == (E, G)
        check(lib.ms_wide_act(ct.byref(pol.mlp_params()), ptr(obs_i8), stride, E, ptr(uniforms), ptr(action),
                              ptr(logprob), stream_ptr(stream)))
        return action, logprob

    def wide_epoch(self, states_i8, actions_i32, old_logprobs, returns_gr, stream=None):
        """The gradient half of one K-epoch step of ``update_wide`` (ms_wide_grad): returns a function
        that writes the epoch's gradient into ``policy``'s .grad tensors and returns the per-group loss."""
        R, G, stride = states_i8.shape
        pol = self.policy
        assert G == pol.G and states_i8.dtype == torch.int8 and states_i8.is_contiguous()
        assert actions_i32.shape == (R, G) and actions_i32.dtype == torch.int32 and actions_i32.is_contiguous()
        assert old_logprobs.shape == (R, G) and old_logprobs.is_contiguous()
        assert returns_gr.shape == (G, R) and returns_gr.is_contiguous()
        for prm in pol.parameters():
            if prm.grad is None:
                prm.grad = torch.zeros_like(prm)
        dev = states_i8.device
        loss_buf = torch.empty((G, 3), dtype=torch.float32, device=dev)
        a = pol.mlp_params()
        c = pol.critic_mlp_params()
        ws_bytes = lib.ms_wide_workspace_bytes(ct.byref(a), R)
        if ws_bytes == 0:
            check(MS_EINVAL)  # raises with ms_last_error()
        # the workspace is cached across updates (same rows / net shape: same plan)
        ws = getattr(self, "_wide_ws", None)
        if ws is None or ws.device != dev or ws.numel() * 4 < ws_bytes:
            ws = self._wide_ws = torch.empty(((ws_bytes + 3) // 4,), dtype=torch.float32, device=dev)
        batch = abi.MsWideBatch(ptr(states_i8), ptr(actions_i32), ptr(old_logprobs), ptr(returns_gr), stride, R)
        grads = abi.MsPpoGrads(*[ptr(getattr(pol, k).grad) for k in ACTOR_KEYS + CRITIC_KEYS], ptr(loss_buf))
        keep = (states_i8, actions_i32, old_logprobs, returns_gr, ws, loss_buf)  # the structs' pointees

        def run():
            assert keep
            # the loss combination reads loss_buf after the kernel: both on the kernel's stream
            with _on_stream(stream):
                check(lib.ms_wide_grad(ct.byref(a), ct.byref(c), ct.byref(batch), ct.c_float(self.eps_clip), ptr(ws),
                                       ws_bytes, ct.byref(grads), stream_ptr(stream)))
                return loss_buf[:, 0] + 0.5 * loss_buf[:, 1] - 0.01 * loss_buf[:, 2]

        return run

    def update_wide(self, states_i8, actions_i32, old_logprobs, returns_gr, stream=None):
        """K epochs of PPO.update (PPOmodules.py:127-174) for the aggregated agents' nets: the gradient
        of each group's mean loss from ms_wide_grad (HIP), all-reduced across ranks when set, then
        the HIP Adam. states_i8 [R, G, stride] int8 rows, actions [R, G] int32, old_logprobs [R, G]
        f32, returns [G, R] f32 normalised (discounted_returns). Returns the K per-group losses."""
        losses = []
        # the gradient zero-init, the kernel, the all-reduce and Adam in one stream order
        with _on_stream(stream):
            epoch = self.wide_epoch(states_i8, actions_i32, old_logprobs, returns_gr, stream)
            for _ in range(self.K):
                loss = epoch()
                if self.allreduce is not None:
                    self.allreduce(self.policy.parameters())
                self.hip_optimizer.step(stream)
                losses.append(loss)
        self.last_losses = losses
        return losses

    @torch.no_grad()
    def sync_old(self):
        """policy_old.load_state_dict(policy.state_dict()) (PPOmodules.py:171): one multi-tensor copy
        launch for all tensors instead of a copy node per tensor (update 8.63 -> 8.59 ms, profiles/r6e)."""
        keys = ACTOR_KEYS + CRITIC_KEYS
        torch._foreach_copy_([getattr(self.policy_old, k).data for k in keys], [getattr(self.policy, k).data for k in keys])

    def update(self, states, actions, old_logprobs, returns):
        """K epochs of full-batch clipped-surrogate PPO (PPOmodules.py:144-168).

        states [G, R, D] float, actions [G, R] int64, old_logprobs [G, R], returns [G, R]
        (already normalised). Each group's loss is the mean over its R rows; the
        groups' losses are summed, so every group receives exactly its own gradient.
        """
        losses = []
        for _ in range(self.K):
            logprobs, values, entropy = self.policy.evaluate(states, actions)
            ratios = torch.exp(logprobs - old_logprobs)
            adv = returns - values.detach()
            surr1 = ratios * adv
            surr2 = torch.clamp(ratios, 1 - self.eps_clip, 1 + self.eps_clip) * adv
            mse = ((values - returns) ** 2).mean(dim=1, keepdim=True)  # nn.MSELoss() per group, broadcast
            loss = -torch.min(surr1, surr2) + 0.5 * mse - 0.01 * entropy
            per_group = loss.mean(dim=1)
            self.optimizer.zero_grad()
            per_group.sum().backward()
            if self.allreduce is not None:
                self.allreduce(self.policy.parameters())
            self.optimizer.step()
            losses.append(per_group.detach())
        self.last_losses = losses
        return losses

    def update_fused(self, states_i8, actions_i8, old_logprobs, returns_teg, unit_of_group, T: int, E: int,
                     stream=None, common_row=None, returns_ld: int = 0, core_owner=None, unit_major: bool = False):
        """The same K epochs with the gradient from the fused HIP kernel (ms_ppo_grad).

        states_i8 [R, U, stride] int8 rollout rows (R = T*E, row r = t*E + e), actions_i8 [R, U],
        old_logprobs [R, U] f32, returns_teg [T, E, G] f32 normalised (unit_returns), unit_of_group [G] int32
        (device). Adam (HIP, ms_adam_step) applies the gradient; with several ranks the gradient is
        all-reduced first. common_row (int8 [stride], device, optional): rows equal to it share one
        forward and one backward pass (same gradient up to f32 summation order). core_owner [R, C]
        (with common_row): states_i8 are compact acceptor rows [R, C, stride] (regen_acceptor_rows).
        unit_major: states_i8 [U, R, stride], actions_i8 / old_logprobs [U, R] instead."""
        epoch = self.fused_epoch(states_i8, actions_i8, old_logprobs, returns_teg, unit_of_group, T, E, stream,
                                 common_row, returns_ld, core_owner, unit_major)
        losses = []
        for _ in range(self.K):
            loss = epoch()
            if self.allreduce is not None:
                self.allreduce(self.policy.parameters())
            self.hip_optimizer.step(stream)
            losses.append(loss)
        self.last_losses = losses
        return losses

    def fused_epoch(self, states_i8, actions_i8, old_logprobs, returns_teg, unit_of_group, T: int, E: int,
                    stream=None, common_row=None, returns_ld: int = 0, core_owner=None, unit_major: bool = False):
        """The gradient half of one K-epoch step of ``update_fused``, for callers that all-reduce
        several groups' gradients in one call (Trainer.update): returns a function that writes this
        epoch's gradient into ``policy``'s .grad tensors (ms_ppo_grad) and returns the per-group loss
        (the Adam step is ``hip_optimizer.step``)."""
        pol = self.policy
        # compact acceptor rows (core_owner [R, C]): states are the core rows [R, C, stride], and U
        # (= N*C units) comes from the actions
        if unit_major:  # [U, R(, stride)]: row (r, u) at u * R + r
            U, R, stride = states_i8.shape
            assert core_owner is None and actions_i8.shape == (U, R) and old_logprobs.shape == (U, R)
        else:
            R, U, stride = states_i8.shape
        n_cores = 0
        if core_owner is not None:
            n_cores, U = U, actions_i8.shape[1]
            assert common_row is not None and core_owner.shape == (R, n_cores) and core_owner.is_contiguous()
        assert R == T * E and states_i8.is_contiguous() and actions_i8.is_contiguous()
        for prm in pol.parameters():
            if prm.grad is None:
                prm.grad = torch.zeros_like(prm)
        loss_buf = torch.empty((pol.G, 3), dtype=torch.float32, device=states_i8.device)
        a = pol.mlp_params()
        c = pol.critic_mlp_params()
        ws_bytes = lib.ms_ppo_workspace_bytes(ct.byref(a), R)
        ws = torch.empty(((ws_bytes + 3) // 4,), dtype=torch.float32, device=states_i8.device)
        batch = abi.MsPpoBatch(ptr(states_i8), ptr(actions_i8), ptr(old_logprobs), ptr(returns_teg),
                               ptr(unit_of_group), stride, T, U, E, ptr(common_row), int(returns_ld),
                               ptr(core_owner), n_cores, int(getattr(self, "row_keys", 0)), R if unit_major else 0)
        grads = abi.MsPpoGrads(*[ptr(getattr(pol, k).grad) for k in ACTOR_KEYS + CRITIC_KEYS], ptr(loss_buf))
        # the structs above hold raw device pointers: the closure keeps every tensor they point into
        # alive until its last launch (a caller's temporaries would otherwise be freed and reused)
        keep = (states_i8, actions_i8, old_logprobs, returns_teg, unit_of_group, common_row, core_owner, ws, loss_buf)

        def launch(out=None):
            """The gradient; the loss terms [G][3] into out (a caller's [G][3] float32 tensor, e.g. one epoch's
            slot of a [n][G][3] buffer whose losses are combined at once) or into this epoch's own buffer."""
            assert keep
            g = grads
            if out is not None:
                assert out.shape == loss_buf.shape and out.dtype == torch.float32 and out.is_contiguous()
                g = abi.MsPpoGrads.from_buffer_copy(grads)
                g.loss = ptr(out)
            check(lib.ms_ppo_grad(ct.byref(a), ct.byref(c), ct.byref(batch), ct.c_float(self.eps_clip), ptr(ws),
                                  ws_bytes, ct.byref(g), stream_ptr(stream)))
            return loss_buf if out is None else out

        def run():
            return combine_losses(launch())

        run.launch = launch
        return run
