"""k_env_step time with and without observation outputs (ms_obs_out pointers NULL skip the
emission), cfg3 at E replicas with random actions. Profiling helper."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ms = importlib.import_module("marl-scheduling_amd")


def timed(env, acts, obs, rew, steps):
    """Device time per step of `steps` env steps replayed from a HIP graph (no host gaps)."""
    for t in range(3):
        env.step(*acts[t], obs=obs, rewards=rew)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for t in range(steps):
            env.step(*acts[t], obs=obs, rewards=rew)
    g.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    g.replay()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1e3 / steps


def main(E=16384, steps=30):
    cfg = ms.abi.named_config("cfg3")
    env = ms.BatchedEnv(cfg, E, seed=0)
    N, C, L, O = env.N, env.C, env.L, env.O
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = []
    for _ in range(steps):
        a = torch.randint(0, O + 1, (E, N, C), device="cuda", generator=g, dtype=torch.int32).to(torch.int8)
        o = torch.randint(0, C + 1, (E, N, L), device="cuda", generator=g, dtype=torch.int32).to(torch.int8)
        p = torch.randint(0, 13, (E, N, L), device="cuda", generator=g, dtype=torch.int32).to(torch.int8)
        acts.append((a, o, p))
    full = env.obs_buffers()
    comp = env.compact_obs_buffers()
    rew = env.reward_buffers()  # preallocated: the loop must not be host-bound
    for name, obs in [("acceptor+offer obs", full), ("offer obs only", dict(offer=full["offer"])),
                      ("offer + compact acceptor", dict(offer=full["offer"], core_rows=comp["core_rows"],
                                                        core_owner=comp["core_owner"])),
                      ("compact acceptor only", dict(core_rows=comp["core_rows"], core_owner=comp["core_owner"])),
                      ("no obs", dict(acceptor=None)), ("acceptor+offer obs", full)]:
        print("%-22s %7.1f us/step" % (name, timed(env, acts, obs, rew, steps)))


if __name__ == "__main__":
    for E in ([int(a) for a in sys.argv[1:]] or [16384]):
        print("E = %d" % E)
        main(E=E)
