"""Loader for libmarlsched.so (the C ABI of include/marlsched.h).

The product has no CPU fallback: if the library is missing or fails to load,
importing this module raises. torch is imported first so that the HIP runtime
torch bundles is the one the library binds to (both carry the soname
libamdhip64.so.7).
"""
from __future__ import annotations

import contextlib
import ctypes as ct
import gc
import os

import torch  # noqa: F401  (load torch's HIP runtime before the library)

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
# MARLSCHED_LIB: an experiment variant built by tools/build_variant.sh (profiling runs only)
LIB_PATH = os.environ.get("MARLSCHED_LIB") or os.path.join(HERE, "libmarlsched.so")


class MarlSchedError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("libmarlsched error %d: %s" % (code, msg))
        self.code = code


ABI_VERSION = 18  # include/marlsched.h MS_ABI_VERSION


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libmarlsched.so is not built (expected at %s); run `python -c 'import __graft_entry__ as g; g.build()'`"
            % LIB_PATH
        )
    L = ct.CDLL(LIB_PATH)
    P = ct.c_void_p
    i32, i64, u32, u64 = ct.c_int32, ct.c_int64, ct.c_uint32, ct.c_uint64
    sig = {
        "ms_last_error": (ct.c_char_p, []),
        "ms_abi_version": (ct.c_int, []),
        "ms_config_shape": (ct.c_int, [ct.POINTER(abi.MsConfig), ct.POINTER(abi.MsShape)]),
        "ms_env_create": (ct.c_int, [ct.POINTER(abi.MsConfig), i64, u64, ct.POINTER(P)]),
        "ms_env_destroy": (None, [P]),
        "ms_env_shape": (ct.c_int, [P, ct.POINTER(abi.MsShape)]),
        "ms_env_reset": (ct.c_int, [P, ct.POINTER(abi.MsObsOut), P]),
        "ms_env_step": (ct.c_int, [P, ct.POINTER(abi.MsActions), ct.POINTER(abi.MsObsOut),
                                   ct.POINTER(abi.MsRewardOut), ct.POINTER(abi.MsEventOut), P]),
        "ms_env_step_act": (ct.c_int, [P, ct.POINTER(abi.MsActions), ct.POINTER(abi.MsObsOut),
                                       ct.POINTER(abi.MsRewardOut), ct.POINTER(abi.MsEventOut),
                                       ct.POINTER(abi.MsFusedAct), P]),
        "ms_env_step_act_supported": (ct.c_int, [P]),
        "ms_env_rollout_act": (ct.c_int, [P, ct.POINTER(abi.MsActions), ct.POINTER(abi.MsObsOut),
                                          ct.POINTER(abi.MsRewardOut), ct.POINTER(abi.MsEventOut),
                                          ct.POINTER(abi.MsFusedAct), ct.POINTER(abi.MsRoundStrides), i32, i32, P]),
        "ms_env_rollout_act_free": (ct.c_int, [P, ct.POINTER(abi.MsActions), ct.POINTER(abi.MsObsOut),
                                               ct.POINTER(abi.MsRewardOut), ct.POINTER(abi.MsEventOut),
                                               ct.POINTER(abi.MsFusedActFree), ct.POINTER(abi.MsRoundStridesFree), i32,
                                               i32, P]),
        "ms_env_rollout_act_free_supported": (ct.c_int, [P]),
        "ms_env_rollout_fill_common": (ct.c_int, [P, ct.POINTER(abi.MsObsOut), ct.POINTER(abi.MsFusedActFree),
                                                  ct.POINTER(abi.MsRoundStridesFree), i32, i32, P]),
        "ms_env_round": (i64, [P]),
        "ms_env_flags": (ct.c_int, [P, ct.POINTER(u32), P]),
        "ms_env_randbelow": (ct.c_int, [P, i64, u32, ct.POINTER(u32), P]),
        "ms_env_auctioneer": (ct.c_int, [P, P, P]),
        "ms_env_get_rng": (ct.c_int, [P, i64, ct.POINTER(u32), ct.POINTER(i32), P]),
        "ms_env_set_rng": (ct.c_int, [P, i64, ct.POINTER(u32), i32, P]),
        "ms_env_export": (ct.c_int, [P, ct.POINTER(abi.MsStateHost), P]),
        "ms_env_import": (ct.c_int, [P, ct.POINTER(abi.MsStateHost), P]),
        "ms_policy_act": (ct.c_int, [ct.POINTER(abi.MsMlpParams), P, i32, i64, i32, i32, u64, u64, P, P, P, P, P]),
        "ms_policy_act_common": (ct.c_int, [ct.POINTER(abi.MsMlpParams), P, i32, i64, i32, i32, P, u64, u64, P, P, P,
                                            P, P]),
        "ms_policy_act_compact": (ct.c_int, [ct.POINTER(abi.MsMlpParams), P, P, i32, i64, i32, i32, i32, P, u64, u64,
                                             P, P, P, P, P]),
        "ms_act_round_free": (ct.c_int, [ct.POINTER(abi.MsMlpParams), ct.POINTER(abi.MsMlpParams), P, i32, i32, i32,
                                         ct.POINTER(abi.MsMlpParams), P, P, i32, i32, i32, i32, P, i64, u64, u64, u64,
                                         P, P, P, P, P, P, P, P, P, ct.POINTER(abi.MsPriceTable), i64, P]),
        "ms_price_table_build": (ct.c_int, [ct.POINTER(abi.MsMlpParams), ct.POINTER(abi.MsPriceTable), P]),
        "ms_act_frag_bytes": (ct.c_size_t, [ct.POINTER(abi.MsMlpParams), i32]),
        "ms_act_prepare": (ct.c_int, [ct.POINTER(abi.MsMlpParams), P, i32, P, P]),
        "ms_offer_act_free": (ct.c_int, [ct.POINTER(abi.MsMlpParams), ct.POINTER(abi.MsMlpParams), P, i32, i64, i32,
                                         i32, i32, u64, u64, P, P, P, P, P, P, P, P, i64, P]),
        "ms_discounted_returns": (ct.c_int, [P, i32, i64, i64, ct.c_double, P, P]),
        "ms_unit_returns": (ct.c_int, [P, i32, i32, i64, i32, P, i32, ct.c_double, P, P]),
        "ms_ppo_workspace_bytes": (ct.c_size_t, [ct.POINTER(abi.MsMlpParams), i64]),
        "ms_ppo_grad": (ct.c_int, [ct.POINTER(abi.MsMlpParams), ct.POINTER(abi.MsMlpParams),
                                   ct.POINTER(abi.MsPpoBatch), ct.c_float, P, ct.c_size_t,
                                   ct.POINTER(abi.MsPpoGrads), P]),
        "ms_aggregate_obs": (ct.c_int, [ct.POINTER(abi.MsConfig), i64, P, P, P, P, P, P]),
        "ms_decode_aggregated": (ct.c_int, [ct.POINTER(abi.MsConfig), i64, P, i32, P, P, P, P]),
        "ms_adam_step": (ct.c_int, [ct.POINTER(abi.MsAdamTensor), i32, ct.POINTER(ct.c_double), i32, i64, ct.c_double,
                                    ct.c_double, ct.c_double, P]),
        "ms_adam_step_dev": (ct.c_int, [ct.POINTER(abi.MsAdamTensor), i32, ct.POINTER(ct.c_double), i32, P,
                                        ct.c_double, ct.c_double, ct.c_double, P]),
        "ms_dqn_act": (ct.c_int, [ct.POINTER(abi.MsQnetParams), P, i32, i64, i32, i32, ct.c_double, P, u64, u64, P,
                                  P, P, P]),
        "ms_regen_agent_rows": (ct.c_int, [ct.POINTER(abi.MsConfig), P, P, P, P, P, i64, P, P, P]),
        "ms_dqn_workspace_bytes": (ct.c_size_t, [ct.POINTER(abi.MsQnetParams), i64]),
        "ms_dqn_grad": (ct.c_int, [ct.POINTER(abi.MsQnetParams), ct.POINTER(abi.MsQnetParams),
                                   ct.POINTER(abi.MsDqnBatch), ct.c_float, P, ct.c_size_t,
                                   ct.POINTER(abi.MsQnetGrads), P]),
        "ms_bdqn_workspace_bytes": (ct.c_size_t, [i32, i32]),
        "ms_bdqn_prepare": (ct.c_int, [ct.POINTER(abi.MsBdqnParams), i32, i32, P, ct.c_size_t, P, P]),
        "ms_bdqn_layer1_scratch_bytes": (ct.c_size_t, [i64, i32]),
        "ms_bdqn_layer1_compact": (ct.c_int, [ct.POINTER(abi.MsBdqnParams), P, P, P, P, i64, i32, i32, i32, i32, P,
                                              ct.c_size_t, P, P]),
        "ms_bdqn_act": (ct.c_int, [ct.POINTER(abi.MsBdqnParams), P, P, i32, P, i64, P, P, P, P]),
        "ms_bdqn_act_compact": (ct.c_int, [ct.POINTER(abi.MsBdqnParams), P, P, P, P, i64, i32, i32, i32, i32, P,
                                           ct.c_size_t, P, P, P, P]),
        "ms_bdqn_update_workspace_bytes": (ct.c_size_t, [ct.POINTER(abi.MsBdqnParams), i32]),
        "ms_bdqn_update": (ct.c_int, [ct.POINTER(abi.MsBdqnParams), ct.POINTER(abi.MsBdqnParams),
                                      ct.POINTER(abi.MsBdqnBatch), ct.c_float, ct.c_float, P, ct.c_size_t,
                                      ct.POINTER(abi.MsBdqnGrads), P]),
        "ms_wide_act": (ct.c_int, [ct.POINTER(abi.MsMlpParams), P, i32, i64, P, P, P, P]),
        "ms_wide_workspace_bytes": (ct.c_size_t, [ct.POINTER(abi.MsMlpParams), i64]),
        "ms_wide_grad": (ct.c_int, [ct.POINTER(abi.MsMlpParams), ct.POINTER(abi.MsMlpParams),
                                    ct.POINTER(abi.MsWideBatch), ct.c_float, P, ct.c_size_t,
                                    ct.POINTER(abi.MsPpoGrads), P]),
    }
    L.ms_abi_version.restype = ct.c_int
    version = L.ms_abi_version()
    # ABI 14 added ms_bdqn_update*, 15 ms_bdqn_act_compact, 16 ms_mlp_params.row_base (a trailing field an
    # older library does not read: its acting draws are those of row_base 0) and ms_env_step_act /
    # ms_env_rollout_act, 17 ms_env_rollout_act_free, 18 its own_action / own_logprob (trailing fields a 17
    # library does not read: it writes the owned items into the rings itself). An older library (an A/B variant built
    # before them, tools/gpu_job.sh ab step) loads without them only when MARLSCHED_LENIENT_ABI=1 asks for it
    lenient = os.environ.get("MARLSCHED_LENIENT_ABI") == "1" and version in (13, 14, 15, 16, 17, 18)
    if version != ABI_VERSION and not lenient:
        raise ImportError("libmarlsched.so ABI version mismatch (%d, want %d)" % (version, ABI_VERSION))
    for name, (res, args) in sig.items():
        if (version < 14 and name.startswith("ms_bdqn_update")) or (version < 15 and name == "ms_bdqn_act_compact") \
                or (version < 16 and (name.startswith("ms_env_step_act") or name == "ms_env_rollout_act")) \
                or (version < 17 and name.startswith("ms_env_rollout_act_free")):
            continue
        if lenient and not hasattr(L, name):  # an older build of this ABI (A/B variants)
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


lib = _load()
ABI_LOADED = int(lib.ms_abi_version())  # < ABI_VERSION only for a lenient load of an older A/B variant


def has(name: str) -> bool:
    """Whether the loaded library exports `name` with its signature set (an older lenient variant may not)."""
    return hasattr(lib, name) and getattr(lib, name).argtypes is not None


# every entry point include/marlsched.h declares (checked by tests)
EXPORTED = (
    "ms_last_error", "ms_abi_version", "ms_config_shape", "ms_env_create", "ms_env_destroy", "ms_env_shape",
    "ms_env_reset", "ms_env_step", "ms_env_step_act", "ms_env_step_act_supported", "ms_env_rollout_act",
    "ms_env_rollout_act_free", "ms_env_rollout_act_free_supported", "ms_env_rollout_fill_common", "ms_env_round", "ms_env_flags", "ms_env_randbelow", "ms_env_auctioneer",
    "ms_env_get_rng", "ms_env_set_rng", "ms_env_export",
    "ms_env_import", "ms_policy_act", "ms_policy_act_common", "ms_policy_act_compact",
    "ms_act_round_free", "ms_price_table_build", "ms_act_frag_bytes", "ms_act_prepare", "ms_offer_act_free", "ms_discounted_returns", "ms_unit_returns",
    "ms_ppo_workspace_bytes", "ms_ppo_grad", "ms_adam_step", "ms_adam_step_dev",
    "ms_aggregate_obs", "ms_decode_aggregated", "ms_dqn_act", "ms_dqn_workspace_bytes", "ms_dqn_grad",
    "ms_regen_agent_rows", "ms_bdqn_workspace_bytes", "ms_bdqn_prepare", "ms_bdqn_layer1_scratch_bytes", "ms_bdqn_layer1_compact",
    "ms_bdqn_act", "ms_bdqn_act_compact", "ms_bdqn_update_workspace_bytes", "ms_bdqn_update", "ms_wide_act", "ms_wide_workspace_bytes",
    "ms_wide_grad",
)


def check(rc: int):
    if rc != 0:
        raise MarlSchedError(rc, (lib.ms_last_error() or b"").decode(errors="replace"))


def ptr(t) -> ct.c_void_p | None:
    """Device pointer of a torch tensor (None passes NULL)."""
    if t is None:
        return None
    return ct.c_void_p(t.data_ptr())


_capture_depth = 0          # hip_capture bodies currently open in this process
_pending_destroy: list = []  # (fn, handle) released while a capture was open, run after it closes


def capturing() -> bool:
    """True inside a hip_capture body or any stream capture on the current stream."""
    if _capture_depth > 0:
        return True
    try:
        return bool(torch.cuda.is_available() and torch.cuda.is_current_stream_capturing())
    except RuntimeError:
        return False


def release(fn, handle) -> None:
    """fn(handle) now, or after the open capture ends: a hipFree inside a global-mode stream capture is an
    operation the capture does not permit and invalidates the graph being recorded (the last reference to
    a BatchedEnv can drop inside a captured body, and its finalizer frees the env's device state)."""
    if capturing():
        _pending_destroy.append((fn, handle))
    else:
        fn(handle)


def drain_released() -> None:
    """Run the releases deferred by captures that have closed."""
    if _capture_depth > 0:
        return
    while _pending_destroy:
        fn, handle = _pending_destroy.pop()
        fn(handle)


@contextlib.contextmanager
def hip_capture(graph, **kw):
    """torch.cuda.graph(graph, **kw) with device frees held off until the capture ends: Python's cyclic
    garbage collector is disabled (a collection would run finalizers inside the capture) and a finalizer
    that still runs there (a refcount drop to zero) queues its free through release()."""
    global _capture_depth
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    _capture_depth += 1
    try:
        with torch.cuda.graph(graph, **kw):
            yield
    finally:
        _capture_depth -= 1
        if was:
            gc.enable()
        drain_released()


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ct.c_void_p(s.cuda_stream)
