"""marl-scheduling_amd — MI355X-native hot path of lr40/marl-scheduling.

The per-round environment step (World.step1 + observations + rewards), the
PPO action selection, the return estimation and the PPO update (fused
forward + clipped-surrogate loss + backward in ``k_ppo_grad``, then ``k_adam``)
run as HIP kernels for gfx950 in libmarlsched.so (C ABI: include/marlsched.h).
PyTorch-ROCm provides device memory, streams, HIP-graph capture and
torch.distributed (RCCL). This package name is not a Python identifier;
import it with ``importlib.import_module("marl-scheduling_amd")``.
"""
from . import abi
from ._lib import LIB_PATH, MarlSchedError, check, lib
from .env import BatchedEnv, decode_accepted, decode_terminated

__all__ = ["abi", "lib", "check", "LIB_PATH", "MarlSchedError", "BatchedEnv", "decode_accepted", "decode_terminated"]
