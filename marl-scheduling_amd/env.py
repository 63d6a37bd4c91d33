"""Batched env replicas on the device (torch tensors in, torch tensors out).

``BatchedEnv`` is the E-replica counterpart of the reference's
``SchedulingEnv.step()/reset()`` (SchedulingEnvironment.py:32-109): E
independent worlds advance one round per ``step`` with one HIP kernel launch
(ms_env_step). Observations are int8 rows, rewards f32/int32, all resident in
HBM; optional ``out=`` tensors let a trainer write straight into its rollout
buffers.
"""
from __future__ import annotations

import ctypes as ct

import numpy as np
import torch

from . import abi
from ._lib import check, drain_released, has, lib, ptr, release, stream_ptr


class BatchedEnv:
    def __init__(self, cfg: abi.MsConfig, n_envs: int, seed: int = 0, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("BatchedEnv needs a HIP device (no CPU fallback)")
        drain_released()  # frees deferred by a capture that was not a hip_capture
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.cfg = cfg
        self.E = int(n_envs)
        self.seed = int(seed)
        self._h = ct.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.ms_env_create(ct.byref(cfg), self.E, ct.c_uint64(self.seed), ct.byref(self._h)))
        sh = abi.MsShape()
        check(lib.ms_env_shape(self._h, ct.byref(sh)))
        self.shape = sh
        self.N, self.C, self.L, self.O = sh.n_agents, sh.n_cores, sh.collection_length, sh.max_offers
        self.free_prices = bool(cfg.free_prices)

    def close(self):
        """ms_env_destroy (deferred to the end of an open HIP-graph capture, _lib.release)."""
        if getattr(self, "_h", None):
            h, self._h = self._h, None
            release(lib.ms_env_destroy, h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- buffers
    def obs_buffers(self, auctioneer=False):
        s, E, d = self.shape, self.E, self.device
        acc = torch.empty((E, self.N, self.C, s.acc_obs_stride), dtype=torch.int8, device=d)
        off = torch.empty((E, self.N, self.L, s.off_obs_stride), dtype=torch.int8, device=d)
        auct = torch.empty((E, self.C, s.acc_obs_stride), dtype=torch.int8, device=d) if auctioneer else None
        return dict(acceptor=acc, offer=off, auctioneer=auct)

    def compact_obs_buffers(self):
        """Compact acceptor observations (ms_obs_out.core_rows / core_owner) + the offer rows."""
        s, E, d = self.shape, self.E, self.device
        return dict(core_rows=torch.empty((E, self.C, s.acc_obs_stride), dtype=torch.int8, device=d),
                    core_owner=torch.empty((E, self.C), dtype=torch.int8, device=d),
                    offer=torch.empty((E, self.N, self.L, s.off_obs_stride), dtype=torch.int8, device=d))

    def reward_buffers(self, aggregated=False):
        E, d = self.E, self.device
        r = dict(
            offer=torch.empty((E, self.N, self.L), dtype=torch.float32, device=d),
            price=torch.empty((E, self.N, self.L), dtype=torch.float32, device=d) if self.free_prices else None,
            acceptor=torch.empty((E, self.N, self.C), dtype=torch.int32, device=d),
            auctioneer=torch.empty((E, self.C), dtype=torch.int32, device=d),
            agent=torch.empty((E, self.N), dtype=torch.int32, device=d),
        )
        if aggregated:  # getAggregatedFixedPricesReward (Reward.py:92-143)
            r["aggregated_offer"] = torch.empty((E, self.N), dtype=torch.int32, device=d)
            r["aggregated_acceptor"] = torch.empty((E, self.N), dtype=torch.int32, device=d)
        return r

    # ---- aggregated agents (Agent.py:73-140, 359-492)
    def aggregated_dims(self):
        """(dim, stride) of the aggregated acceptor, offer and fully aggregated rows."""
        N, C, L, d_acc = self.N, self.C, self.L, self.shape.acc_obs_dim
        dims = dict(acceptor=C * d_acc, offer=2 * C + 2 * L, fully=2 * C + 2 * L + C * d_acc)
        return {k: (v, (v + 3) // 4 * 4) for k, v in dims.items()}

    def aggregated_action_counts(self):
        """(O+1)^C acceptor and (C+1)^L offer actions per agent (PPOmodules.py:180, 198)."""
        return (self.O + 1) ** self.C, (self.C + 1) ** self.L

    def aggregate_obs(self, obs, out=None, kinds=("acceptor", "offer"), stream=None):
        """Aggregated observations [E, N, stride] int8 from the divided ones (ms_aggregate_obs)."""
        dims = self.aggregated_dims()
        if out is None:
            out = {k: torch.empty((self.E, self.N, dims[k][1]), dtype=torch.int8, device=self.device) for k in kinds}
        for k, t in out.items():
            assert t.dtype == torch.int8 and t.is_contiguous() and t.numel() == self.E * self.N * dims[k][1], k
        check(lib.ms_aggregate_obs(ct.byref(self.cfg), self.E, ptr(obs["acceptor"]), ptr(obs["offer"]),
                                   ptr(out.get("acceptor")), ptr(out.get("offer")), ptr(out.get("fully")),
                                   stream_ptr(stream)))
        return out

    def decode_aggregated(self, numbers, fully: bool, acceptor=None, offer_core=None, n_bad=None, stream=None):
        """Agent action numbers (int32: [2, E, N] acceptor/offer numbers, or [E, N] fully aggregated)
        -> divided actions (int8 [E, N, C], [E, N, L]) for step (ms_decode_aggregated)."""
        assert numbers.dtype == torch.int32 and numbers.is_contiguous()
        assert numbers.numel() == self.E * self.N * (1 if fully else 2)
        if acceptor is None:
            acceptor = torch.empty((self.E, self.N, self.C), dtype=torch.int8, device=self.device)
        if offer_core is None:
            offer_core = torch.empty((self.E, self.N, self.L), dtype=torch.int8, device=self.device)
        check(lib.ms_decode_aggregated(ct.byref(self.cfg), self.E, ptr(numbers), int(bool(fully)), ptr(acceptor),
                                       ptr(offer_core), ptr(n_bad), stream_ptr(stream)))
        return acceptor, offer_core

    def regen_agent_rows(self, core_rows, core_owner, slot_pairs, frame, agent, acceptor=None, offer=None,
                         stream=None):
        """ms_regen_agent_rows: aggregated acceptor / offer rows of (record frame[b], agent[b]) from compact
        records core_rows [M, C, acc_stride], core_owner [M, C], slot_pairs [M, N, L, 2] (int8)."""
        n = frame.numel()
        assert frame.dtype == torch.int64 and agent.dtype == torch.int32 and agent.numel() == n
        d = self.aggregated_dims()
        if acceptor is None and offer is None:
            acceptor = torch.empty((n, d["acceptor"][1]), dtype=torch.int8, device=self.device)
            offer = torch.empty((n, d["offer"][1]), dtype=torch.int8, device=self.device)
        check(lib.ms_regen_agent_rows(ct.byref(self.cfg), ptr(core_rows), ptr(core_owner), ptr(slot_pairs), ptr(frame),
                                      ptr(agent), n, ptr(acceptor), ptr(offer), stream_ptr(stream)))
        return acceptor, offer

    def event_buffers(self):
        E, d = self.E, self.device
        return dict(
            accepted=torch.empty((E, self.C, abi.ACCEPT_REC_BYTES), dtype=torch.int8, device=d),
            terminated=torch.empty((E, self.C, abi.TERM_REC_BYTES), dtype=torch.int8, device=d),
        )

    def metrics_buffer(self, slots: int = 1):
        """Episode accumulators [slots][E] of ms_env_metrics (zeroed), for events["metrics"]:
        round r adds into slot (r // episode_length) % slots."""
        return torch.zeros((slots, self.E, abi.METRICS_BYTES), dtype=torch.uint8, device=self.device)

    # ---- API
    @property
    def round(self) -> int:
        return int(lib.ms_env_round(self._h))

    def reset(self, obs=None, stream=None):
        """SchedulingEnv.reset (SchedulingEnvironment.py:85-109): observations only."""
        obs = obs or self.obs_buffers()
        o = abi.MsObsOut(ptr(obs.get("acceptor")), ptr(obs.get("offer")), ptr(obs.get("auctioneer")),
                         ptr(obs.get("core_rows")), ptr(obs.get("core_owner")))
        check(lib.ms_env_reset(self._h, ct.byref(o), stream_ptr(stream)))
        return obs

    def step(self, acceptor, offer_core, offer_price=None, auctioneer=None, obs=None, rewards=None, events=None,
             stream=None, next_act=None):
        """One round of SchedulingEnv.step (SchedulingEnvironment.py:32-83) for all replicas.

        acceptor [E,N,C] int8, offer_core [E,N,L] int8, offer_price [E,N,L] int8
        (free prices), auctioneer [E,C] int8 or None for the in-kernel
        HardcodedAuctioneerAcceptor. Returns (obs, rewards, events) dicts.
        next_act (an abi.MsFusedAct): the next round's acting fused into the round (ms_env_step_act; fixed
        prices, compact acceptor observations; see fused_act_supported).
        """
        for t in (acceptor, offer_core, offer_price, auctioneer):
            if t is not None:
                assert t.dtype == torch.int8 and t.is_contiguous() and t.device == self.device
        # acceptor and offer_core both None: the hard-coded agents act in the kernel (fixed prices)
        assert (acceptor is None) == (offer_core is None)
        if acceptor is not None:
            assert acceptor.numel() == self.E * self.N * self.C and offer_core.numel() == self.E * self.N * self.L
        if self.free_prices:
            assert offer_price is not None and offer_price.numel() == self.E * self.N * self.L
        if auctioneer is not None:
            assert auctioneer.numel() == self.E * self.C
        obs = self.obs_buffers() if obs is None else obs
        rewards = self.reward_buffers() if rewards is None else rewards
        a, o, r, ev = self._step_structs(acceptor, offer_core, offer_price, auctioneer, obs, rewards, events)
        if next_act is not None:
            check(lib.ms_env_step_act(self._h, ct.byref(a), ct.byref(o), ct.byref(r), ct.byref(ev) if ev else None,
                                      ct.byref(next_act), stream_ptr(stream)))
        else:
            check(lib.ms_env_step(self._h, ct.byref(a), ct.byref(o), ct.byref(r), ct.byref(ev) if ev else None,
                                  stream_ptr(stream)))
        return obs, rewards, events

    @staticmethod
    def check_rings(rings, n_rounds: int):
        """The bounds contract of the one-launch rollouts (marlsched.h): each (tensor, stride, dtype) is a ring's
        round-0 slot, read or written again at stride bytes for every later round, so its storage must hold
        n_rounds slots (the kernel sees pointers only: a short ring would be an out-of-bounds GPU access)."""
        for t, stride, dtype in rings:
            if t is None:
                continue
            assert t.is_cuda and t.is_contiguous() and t.dtype == dtype, (t.shape, t.dtype, dtype)
            st = t.untyped_storage()
            end = st.data_ptr() + st.nbytes()
            assert stride >= 0 and (stride == 0 or stride >= t.numel() * t.element_size()), "overlapping ring slots"
            last = t.data_ptr() + (int(n_rounds) - 1) * int(stride) + t.numel() * t.element_size()
            assert last <= end, "ring holds fewer than n_rounds slots at its stride"

    def _ring_list(self, acceptor, offer_core, obs, rewards, strides, price=False):
        i8, i32, f32 = torch.int8, torch.int32, torch.float32
        rings = [(acceptor, strides.acceptor_action, i8), (offer_core, strides.offer_action, i8),
                 (obs.get("core_rows"), strides.core_rows, i8), (obs.get("core_owner"), strides.core_owner, i8),
                 (obs.get("offer"), strides.offer_obs, i8), (rewards.get("offer"), strides.offer_reward, f32),
                 (rewards.get("acceptor"), strides.acceptor_reward, i32),
                 (rewards.get("agent"), strides.agent_reward, i32),
                 (rewards.get("auctioneer"), strides.auctioneer_reward, i32)]
        if price:
            rings.append((rewards.get("price"), strides.price_reward, f32))
        return rings

    def rollout_act(self, acceptor, offer_core, obs, rewards, next_act, strides, n_rounds, act_after_last=False,
                    events=None, stream=None, next_out=None):
        """n_rounds rounds of step(next_act=...) in one launch (ms_env_rollout_act): round t reads and
        writes the given arrays advanced by t * strides (an abi.MsRoundStrides, bytes) and acts with the
        Philox offsets + t * strides.offset_step. Bit-identical to the n_rounds step calls.
        next_out: the tensors behind next_act's outputs, dict(off_action, off_logprob, acc_action, acc_logprob)
        (round 0's slots), bounds-checked like the other rings when given."""
        for t in (acceptor, offer_core):
            assert t.dtype == torch.int8 and t.device == self.device
        rings = self._ring_list(acceptor, offer_core, obs, rewards, strides)
        if next_out is not None and (n_rounds > 1 or act_after_last):
            n_act = n_rounds if act_after_last else n_rounds - 1
            self.check_rings([(next_out["off_action"], strides.next_off_action, torch.int8),
                              (next_out["off_logprob"], strides.next_off_logprob, torch.float32),
                              (next_out["acc_action"], strides.next_acc_action, torch.int8),
                              (next_out["acc_logprob"], strides.next_acc_logprob, torch.float32)], n_act)
        self.check_rings(rings, n_rounds)
        a, o, r, ev = self._step_structs(acceptor, offer_core, None, None, obs, rewards, events)
        check(lib.ms_env_rollout_act(self._h, ct.byref(a), ct.byref(o), ct.byref(r), ct.byref(ev) if ev else None,
                                     ct.byref(next_act), ct.byref(strides), int(n_rounds), int(bool(act_after_last)),
                                     stream_ptr(stream)))

    def rollout_act_free(self, acceptor, offer_core, obs, rewards, next_act, next_out, strides, n_rounds,
                         act_after_last=False, events=None, stream=None):
        """A locally shared free-price rollout of n_rounds rounds in one launch (ms_env_rollout_act_free; BASELINE
        cfg3): round t steps the replicas with the actions advanced by t strides and next_out["env_price"] as the
        offer prices, writes obs / rewards advanced by t strides, then samples round t + 1's actions into next_act's
        outputs (an abi.MsFusedActFree; next_out: its tensors, round 0's slots) advanced by t strides. Bit-identical
        to n_rounds pairs of step + act_round_free (SchedulingEnvironment.py:150-172, trainPPO.py:160-167)."""
        i8, f32 = torch.int8, torch.float32
        assert self.free_prices and next_out["env_price"].numel() == self.E * self.N * self.L
        rings = self._ring_list(acceptor, offer_core, obs, rewards, strides, price=True)
        rings.append((next_out["env_price"], 0, i8))
        self.check_rings(rings, n_rounds)
        if n_rounds > 1 or act_after_last:
            n_act = n_rounds if act_after_last else n_rounds - 1
            self.check_rings([(next_out["core_action"], strides.next_core_action, i8),
                              (next_out["core_logprob"], strides.next_core_logprob, f32),
                              (next_out["price_state"], strides.next_price_state, i8),
                              (next_out["price_action"], strides.next_price_action, i8),
                              (next_out["price_logprob"], strides.next_price_logprob, f32),
                              (next_out["acc_action"], strides.next_acc_action, i8),
                              (next_out["acc_logprob"], strides.next_acc_logprob, f32)], n_act)
            if next_out.get("own_action") is not None:  # the owned items by core [E][C] (ABI 18)
                assert next_out["own_action"].numel() == self.E * self.C
                self.check_rings([(next_out["own_action"], strides.next_own_action, i8),
                                  (next_out["own_logprob"], strides.next_own_logprob, f32)], n_act)
        assert bool(next_act.own_action) == (next_out.get("own_action") is not None)
        a, o, r, ev = self._step_structs(acceptor, offer_core, next_out["env_price"], None, obs, rewards, events)
        check(lib.ms_env_rollout_act_free(self._h, ct.byref(a), ct.byref(o), ct.byref(r),
                                          ct.byref(ev) if ev else None, ct.byref(next_act), ct.byref(strides),
                                          int(n_rounds), int(bool(act_after_last)), stream_ptr(stream)))

    def fill_common(self, obs, next_act, strides, n_rounds, act_after_last=False, stream=None):
        """The acceptor items of cores their agent does not own that rollout_act_free(next_act.defer_common = 1)
        left (ms_env_rollout_fill_common): the same obs / strides / next_act as that call, with next_act.offset_dev
        holding the offsets it held then."""
        o = abi.MsObsOut(None, None, None, None, ptr(obs.get("core_owner")))
        check(lib.ms_env_rollout_fill_common(self._h, ct.byref(o), ct.byref(next_act), ct.byref(strides), int(n_rounds),
                                             int(bool(act_after_last)), stream_ptr(stream)))

    def rollout_free_supported(self) -> bool:
        """Whether rollout_act_free can run this env's rounds (ms_env_rollout_act_free_supported)."""
        return has("ms_env_rollout_act_free_supported") and bool(lib.ms_env_rollout_act_free_supported(self._h))

    def _step_structs(self, acceptor, offer_core, offer_price, auctioneer, obs, rewards, events):
        a = abi.MsActions(ptr(acceptor), ptr(offer_core), ptr(offer_price if self.free_prices else None),
                          ptr(auctioneer))
        o = abi.MsObsOut(ptr(obs.get("acceptor")), ptr(obs.get("offer")), ptr(obs.get("auctioneer")),
                         ptr(obs.get("core_rows")), ptr(obs.get("core_owner")))
        r = abi.MsRewardOut(ptr(rewards.get("offer")), ptr(rewards.get("price")), ptr(rewards.get("acceptor")),
                            ptr(rewards.get("auctioneer")), ptr(rewards.get("agent")),
                            ptr(rewards.get("aggregated_offer")), ptr(rewards.get("aggregated_acceptor")))
        ev = None
        if events:
            m = events.get("metrics")
            if m is not None:
                assert m.dtype == torch.uint8 and m.is_contiguous() and m.shape[1:] == (self.E, abi.METRICS_BYTES)
            ev = abi.MsEventOut(ptr(events.get("accepted")), ptr(events.get("terminated")),
                                ptr(events.get("launch_span")), ptr(m), 0 if m is None else m.shape[0])
        return a, o, r, ev

    def fused_act_supported(self) -> bool:
        """Whether step(next_act=...) can run this env's rounds (ms_env_step_act_supported; False for an older
        library without it)."""
        return has("ms_env_step_act_supported") and bool(lib.ms_env_step_act_supported(self._h))

    def flags(self, stream=None) -> int:
        f = ct.c_uint32()
        check(lib.ms_env_flags(self._h, ct.byref(f), stream_ptr(stream)))
        return int(f.value)

    def randbelow(self, n: int, env_index: int = 0, stream=None) -> int:
        """random._randbelow(n) on replica env_index's stream (random.randint(a, b) = a + randbelow(b-a+1))."""
        out = ct.c_uint32()
        check(lib.ms_env_randbelow(self._h, int(env_index), int(n), ct.byref(out), stream_ptr(stream)))
        return int(out.value)

    def auctioneer(self, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        """Auctioneer.getAuctioneerAction (Auctioneer.py:95-102) on the current state of every
        replica: int8 [E, C] actions (O = reject); consumes the tie-break draws."""
        if out is None:
            out = torch.empty((self.E, self.C), dtype=torch.int8, device=self.device)
        assert out.dtype == torch.int8 and out.is_contiguous() and out.numel() == self.E * self.C
        check(lib.ms_env_auctioneer(self._h, ptr(out), stream_ptr(stream)))
        return out

    def get_rng_state(self, env_index: int = 0, stream=None):
        """(624 MT19937 words as a tuple of ints, index): the random.getstate() internal state."""
        words = (ct.c_uint32 * 624)()
        idx = ct.c_int32()
        check(lib.ms_env_get_rng(self._h, int(env_index), words, ct.byref(idx), stream_ptr(stream)))
        return tuple(int(w) for w in words), int(idx.value)

    def set_rng_state(self, words, index: int, env_index: int = 0, stream=None):
        buf = (ct.c_uint32 * 624)(*[int(w) for w in words])
        check(lib.ms_env_set_rng(self._h, int(env_index), buf, int(index), stream_ptr(stream)))

    # ---- state export / import (canonical ms_state_host layout)
    def _state_arrays(self):
        E, N, C, L, cap = self.E, self.N, self.C, self.L, self.shape.liability_cap
        return dict(
            round=np.zeros(E, np.int32), flags=np.zeros(E, np.uint32),
            core_owner=np.zeros((E, C), np.int32), core_kind=np.zeros((E, C), np.int32),
            core_rem=np.zeros((E, C), np.int32), core_birth=np.zeros((E, C), np.int32),
            slot_kind=np.zeros((E, N, L), np.int32), slot_rem=np.zeros((E, N, L), np.int32),
            slot_wait=np.zeros((E, N, L), np.int32), slot_birth=np.zeros((E, N, L), np.int32),
            offer_core=np.zeros((E, N, L), np.int32), offer_recip=np.zeros((E, N, L), np.int32),
            offer_price=np.zeros((E, N, L), np.int32), liab_n=np.zeros((E, C), np.int32),
            liab=np.zeros((E, C, cap, 5), np.int32), mt=np.zeros((E, 624), np.uint32),
            mt_index=np.zeros(E, np.int32),
        )

    @staticmethod
    def _struct(arrs):
        st = abi.MsStateHost()
        for name, _ in abi.MsStateHost._fields_:
            setattr(st, name, arrs[name].ctypes.data)
        return st

    def export_state(self, stream=None) -> dict:
        arrs = self._state_arrays()
        check(lib.ms_env_export(self._h, ct.byref(self._struct(arrs)), stream_ptr(stream)))
        return arrs

    def import_state(self, state: dict, stream=None):
        arrs = self._state_arrays()
        for k, v in arrs.items():
            if k in state:
                v[...] = np.asarray(state[k]).reshape(v.shape).astype(v.dtype)
        check(lib.ms_env_import(self._h, ct.byref(self._struct(arrs)), stream_ptr(stream)))


def decode_accepted(raw: torch.Tensor) -> np.ndarray:
    """[E,C,16] int8 ms_accept_rec bytes -> numpy structured array."""
    dt = np.dtype([("valid", "i1"), ("offerer", "i1"), ("recipient", "i1"), ("slot", "i1"), ("price", "i1"),
                   ("nec_time", "i1"), ("prio", "i1"), ("kind", "i1"), ("order", "i1"), ("pad", "i1", 3),
                   ("round", "<i4")])
    return raw.cpu().numpy().view(dt)[..., 0]


def decode_terminated(raw: torch.Tensor) -> np.ndarray:
    dt = np.dtype([("valid", "i1"), ("owner", "i1"), ("prio", "i1"), ("init_len", "i1"), ("dwell", "<i4")])
    return raw.cpu().numpy().view(dt)[..., 0]
