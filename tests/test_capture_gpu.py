"""Device frees inside a HIP-graph capture are deferred to the capture's end (_lib.release).

Round 3 saw `hipErrorStreamCaptureInvalidated` when a BatchedEnv's finalizer (ms_env_destroy ->
hipFree) ran inside a global-mode capture, followed by `hipErrorStreamCaptureUnsupported` in later
tests. Here the last reference to an env is dropped inside a captured body on purpose: the capture
must stay valid, the free must run once the capture closes, and the graph must replay the same
rounds an eager twin env computes.
"""
import gc

import pytest
import torch

pytestmark = pytest.mark.gpu


def _actions(ms, env, T, seed):
    g = torch.Generator(device=env.device).manual_seed(seed)
    E, N, C, L, O = env.E, env.N, env.C, env.L, env.O
    acc = torch.randint(0, O + 1, (T, E, N, C), device=env.device, generator=g, dtype=torch.int32).to(torch.int8)
    off = torch.randint(0, C + 1, (T, E, N, L), device=env.device, generator=g, dtype=torch.int32).to(torch.int8)
    return acc, off


def test_env_released_inside_capture_is_deferred(ms):
    from importlib import import_module

    lib = import_module("marl-scheduling_amd._lib")
    cfg = ms.abi.named_config("cfg2")
    E, T = 256, 4
    env = ms.BatchedEnv(cfg, E, seed=11)
    twin = ms.BatchedEnv(cfg, E, seed=11)
    doomed = ms.BatchedEnv(cfg, 64, seed=3)
    acc, off = _actions(ms, env, T + 1, 5)
    obs, rew = env.obs_buffers(), env.reward_buffers()
    # one eager round first (the capture records rounds 1..T)
    env.step(acc[0], off[0], obs=obs, rewards=rew)
    twin.step(acc[0], off[0])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    freed_inside = []
    with lib.hip_capture(g):
        for t in range(1, T + 1):
            env.step(acc[t], off[t], obs=obs, rewards=rew)
            if t == 2:
                del doomed  # the last reference: __del__ -> close -> release(ms_env_destroy) inside the capture
                freed_inside.append(len(lib._pending_destroy))
    assert freed_inside == [1], "the free was not deferred inside the capture"
    assert not lib._pending_destroy, "the deferred free did not run when the capture closed"
    gc.collect()
    g.replay()
    for t in range(1, T + 1):
        o_tw, r_tw, _ = twin.step(acc[t], off[t])
    torch.cuda.synchronize()
    assert torch.equal(obs["acceptor"], o_tw["acceptor"]) and torch.equal(obs["offer"], o_tw["offer"])
    for k in ("offer", "acceptor", "auctioneer", "agent"):
        assert torch.equal(rew[k], r_tw[k]), k
    assert env.round == twin.round == T + 1
    # later captures on the same process still work (round 3 saw CaptureUnsupported cascades)
    g2 = torch.cuda.CUDAGraph()
    x = torch.zeros(16, device=env.device)
    with lib.hip_capture(g2):
        x.add_(1.0)
    g2.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 1.0
