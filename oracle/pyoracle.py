"""ctypes loader for the C restatement (oracle/libms_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package. It shares only the
struct layouts of include/marlsched.h (marl-scheduling_amd/abi.py, loaded by
file path so that the product library is never loaded from here).
"""
from __future__ import annotations

import ctypes as ct
import importlib.util
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libms_oracle.so")


def _load_abi():
    spec = importlib.util.spec_from_file_location("_ms_abi_for_oracle", os.path.join(REPO, "marl-scheduling_amd", "abi.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


abi = _load_abi()


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "ms_oracle.c")):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ct.CDLL(LIB_PATH)
        P = ct.c_void_p
        L.mso_create.restype = P
        L.mso_create.argtypes = [P, ct.c_uint64]  # any ms_config-layout struct (product or oracle copy)
        L.mso_destroy.argtypes = [P]
        L.mso_step.argtypes = [P, P, P, P, P, P]
        L.mso_step.restype = ct.c_int
        L.mso_auctioneer_actions.argtypes = [P, P]
        L.mso_observe.argtypes = [P, P, P, P, P, P]
        L.mso_export.argtypes = [P, ct.POINTER(abi.MsStateHost)]
        L.mso_import.argtypes = [P, ct.POINTER(abi.MsStateHost)]
        L.mso_round.restype = ct.c_int64
        L.mso_round.argtypes = [P]
        L.mso_flags.restype = ct.c_uint32
        L.mso_flags.argtypes = [P]
        L.mso_genrand.restype = ct.c_uint32
        L.mso_genrand.argtypes = [P]
        L.mso_random.restype = ct.c_double
        L.mso_random.argtypes = [P]
        L.mso_randbelow.restype = ct.c_uint32
        L.mso_randbelow.argtypes = [P, ct.c_uint32]
        L.mso_mt_seed_words.argtypes = [ct.c_uint64, P, P]
        L.mso_step_batch.argtypes = [P, ct.c_int64, P, P, P, P, P, ct.c_int32, ct.c_int32, P, P, P, ct.c_int]
        L.mso_step_batch.restype = ct.c_int
        _lib = L
    return _lib


class _StepOut(ct.Structure):
    _fields_ = [
        ("offer", ct.c_void_p),
        ("price", ct.c_void_p),
        ("acceptor", ct.c_void_p),
        ("auctioneer", ct.c_void_p),
        ("agent", ct.c_void_p),
        ("termination_revenue", ct.c_int64),
        ("accepted", ct.c_void_p),
        ("terminated", ct.c_void_p),
        ("quality", ct.c_void_p),
        ("n_quality", ct.c_int32),
    ]


def _p(a: np.ndarray):
    return a.ctypes.data_as(ct.c_void_p) if a is not None else None


ACCEPT_DTYPE = np.dtype([("valid", "i1"), ("offerer", "i1"), ("recipient", "i1"), ("slot", "i1"),
                         ("price", "i1"), ("nec_time", "i1"), ("prio", "i1"), ("kind", "i1"),
                         ("order", "i1"), ("pad", "i1", 3), ("round", "<i4")])
TERM_DTYPE = np.dtype([("valid", "i1"), ("owner", "i1"), ("prio", "i1"), ("init_len", "i1"), ("dwell", "<i4")])


def state_arrays(E, N, C, L, cap):
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


def state_struct(arrs: dict) -> abi.MsStateHost:
    st = abi.MsStateHost()
    for name, _ in abi.MsStateHost._fields_:
        a = arrs[name]
        assert a.flags["C_CONTIGUOUS"]
        setattr(st, name, a.ctypes.data)
    return st


class OracleEnv:
    """One env (E = 1) of the C restatement."""

    def __init__(self, cfg: abi.MsConfig, seed: int):
        self.cfg = cfg
        self.shape = abi.config_shape(cfg)
        self.N, self.C, self.L, self.O = (self.shape[k] for k in ("N", "C", "L", "O"))
        self.cap = self.shape["liability_cap"]
        self._cfg_ref = cfg
        self.h = lib().mso_create(ct.addressof(cfg), ct.c_uint64(seed))
        if not self.h:
            raise ValueError("invalid config")

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            lib().mso_destroy(h)
            self.h = None

    @property
    def round(self):
        return lib().mso_round(self.h)

    @property
    def flags(self):
        return lib().mso_flags(self.h)

    def auctioneer_actions(self):
        out = np.zeros(self.C, np.int32)
        lib().mso_auctioneer_actions(self.h, _p(out))
        return out

    def step(self, acc, off_core, off_price=None, auct=None):
        N, C, L = self.N, self.C, self.L
        acc = np.ascontiguousarray(acc, np.int32).reshape(N, C)
        off_core = np.ascontiguousarray(off_core, np.int32).reshape(N, L)
        if off_price is not None:
            off_price = np.ascontiguousarray(off_price, np.int32).reshape(N, L)
        if auct is not None:
            auct = np.ascontiguousarray(auct, np.int32).reshape(C)
        r = dict(
            offer=np.zeros((N, L), np.float64), price=np.zeros((N, L), np.float64),
            acceptor=np.zeros((N, C), np.int64), auctioneer=np.zeros(C, np.int64),
            agent=np.zeros(N, np.int64), accepted=np.zeros(C, ACCEPT_DTYPE),
            terminated=np.zeros(C, TERM_DTYPE), quality=np.zeros(C, np.float64),
        )
        out = _StepOut(_p(r["offer"]), _p(r["price"]), _p(r["acceptor"]), _p(r["auctioneer"]), _p(r["agent"]), 0,
                       _p(r["accepted"]), _p(r["terminated"]), _p(r["quality"]), 0)
        rc = lib().mso_step(self.h, _p(acc), _p(off_core), _p(off_price), _p(auct), ct.byref(out))
        if rc != 0:
            raise RuntimeError("mso_step failed")
        r["termination_revenue"] = out.termination_revenue
        r["quality"] = r["quality"][: out.n_quality].copy()
        return r

    def observe(self):
        N, C, L, O = self.N, self.C, self.L, self.O
        acc = np.zeros((N, C, 3 + 2 * O), np.int32)
        ids = np.zeros((N, C, O), np.int32)
        off = np.zeros((N, L, 2 * C + 2), np.int32)
        auct = np.zeros((C, 3 + 2 * O), np.int32)
        auct_ids = np.zeros((C, O), np.int32)
        lib().mso_observe(self.h, _p(acc), _p(ids), _p(off), _p(auct), _p(auct_ids))
        return dict(acceptor=acc, acceptor_ids=ids, offer=off, auctioneer=auct, auctioneer_ids=auct_ids)

    def export_state(self):
        arrs = state_arrays(1, self.N, self.C, self.L, self.cap)
        lib().mso_export(self.h, ct.byref(state_struct(arrs)))
        return {k: v[0] for k, v in arrs.items()}

    def import_state(self, st: dict):
        arrs = state_arrays(1, self.N, self.C, self.L, self.cap)
        for k in arrs:
            if k in st:
                arrs[k][0] = np.asarray(st[k]).astype(arrs[k].dtype)
        rc = lib().mso_import(self.h, ct.byref(state_struct(arrs)))
        if rc != 0:
            raise ValueError("import rejected")

    def genrand(self):
        return lib().mso_genrand(self.h)

    def random(self):
        return lib().mso_random(self.h)

    def randbelow(self, n):
        return lib().mso_randbelow(self.h, n)


def mt_seed_state(seed: int):
    st = np.zeros(624, np.uint32)
    idx = np.zeros(1, np.int32)
    lib().mso_mt_seed_words(ct.c_uint64(seed), _p(st), _p(idx))
    return st, int(idx[0])


class OracleBatch:
    """E independent oracle envs stepped with device-ABI-shaped int8 actions."""

    def __init__(self, cfg, n_envs, seed):
        self.envs = [OracleEnv(cfg, seed + e) for e in range(n_envs)]
        self.E = n_envs
        self.shape = self.envs[0].shape
        self._ptrs = (ct.c_void_p * n_envs)(*[e.h for e in self.envs])

    def step(self, acc, off_core, off_price=None, threads=1, want_obs=True):
        s = self.shape
        E, N, C, L = self.E, s["N"], s["C"], s["L"]
        acc = np.ascontiguousarray(acc, np.int8)
        off_core = np.ascontiguousarray(off_core, np.int8)
        off_price = None if off_price is None else np.ascontiguousarray(off_price, np.int8)
        acc_obs = np.zeros((E, N, C, s["acc_obs_stride"]), np.int8) if want_obs else None
        off_obs = np.zeros((E, N, L, s["off_obs_stride"]), np.int8) if want_obs else None
        orew = np.zeros((E, N, L), np.float32)
        prew = np.zeros((E, N, L), np.float32)
        arew = np.zeros((E, N, C), np.int32)
        lib().mso_step_batch(self._ptrs, E, _p(acc), _p(off_core), _p(off_price), _p(acc_obs), _p(off_obs),
                             s["acc_obs_stride"], s["off_obs_stride"], _p(orew), _p(prew), _p(arew), threads)
        return dict(acc_obs=acc_obs, off_obs=off_obs, offer=orew, price=prew, acceptor=arew)
