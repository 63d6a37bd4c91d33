"""marl-scheduling_amd — MI355X-native hot path of lr40/marl-scheduling.

The per-round environment step (World.step1 + observations + rewards), the
PPO action selection and the return estimation run as HIP kernels for gfx950
in libmarlsched.so (C ABI: include/marlsched.h); the PPO update runs in
PyTorch-ROCm on the same device. This package name is not a Python
identifier; import it with ``importlib.import_module("marl-scheduling_amd")``.
"""
from . import abi
from ._lib import LIB_PATH, MarlSchedError, check, lib
from .env import BatchedEnv, decode_accepted, decode_terminated

__all__ = ["abi", "lib", "check", "LIB_PATH", "MarlSchedError", "BatchedEnv", "decode_accepted", "decode_terminated"]
