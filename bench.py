#!/usr/bin/env python3
"""Headline benchmark: agent-env-steps/s of the marl-scheduling PPO loop (BASELINE.json cfg3).

One benchmark step = one PPO iteration of the batched trainer: UPDATE_STEP (200)
rounds of policy act (HIP) -> env step (HIP) -> buffer writes, followed by the
full PPO update of every unit type (returns on HIP, K epochs of Adam in
PyTorch-ROCm). Workload per GPU: 16384 env replicas x 8 agents x 8 cores,
collectionLength 3, free prices + commercial reward, locally shared PPO
(SURVEY.md §8(d) cfg3). value = agents x replicas x rounds over all ranks /
max-over-ranks wall time of the timed steps (weak scaling: replicas per GPU fixed).

Run: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run, or
bench.py --gpus N alone, which starts the N rank processes itself (one rank per GPU, RCCL
all-reduce of the shared nets' gradients). The line also carries the env step kernel alone
(pre-sampled actions, seeds {0,1,2}) as "step_kernel".
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

METRIC = "agent-env-steps/sec (whole node), 8 agents×8 cores×16384 envs, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def env_round_bytes(shape, k_new_jobs: int, free: bool, compact: bool = False) -> int:
    """Algorithmic bytes of one env replica's round: SURVEY.md §8(d)'s judge figure,
    B = B_state + B_act + B_obs + B_rew (+ B_liab),
      B_state = 2 (4C + 8NL + 4)          compact state read + write
      B_act   = NC + NL (+ NL free)        actions read
      B_obs   = NC D_acc + NL D_off + C D_acc at 1 B per element (the observations the round hands
                the agents and the auctioneer, whatever form the kernel writes them in: with
                ``compact`` the acceptor rows go out as C owner rows + owners and are regenerated
                where they are read, so the kernel writes fewer bytes than it delivers)
      B_rew   = 4 (NL (1 or 2) + NC + N + C)
    B_liab (16 B per accepted offer) is data dependent and left out: a lower bound. k_new_jobs and
    compact do not change the figure (kept for the callers)."""
    N, C, L = shape.n_agents, shape.n_cores, shape.collection_length
    d_acc, d_off = shape.acc_obs_dim, shape.off_obs_dim
    b_state = 2 * (4 * C + 8 * N * L + 4)
    b_act = N * C + N * L * (2 if free else 1)
    b_obs = N * C * d_acc + N * L * d_off + C * d_acc
    b_rew = 4 * (N * L * (2 if free else 1) + N * C + N + C)
    return b_state + b_act + b_obs + b_rew


def act_out_bytes(shape, free: bool) -> int:
    """Bytes one replica's acting writes per round, the rollout buffers of selectAction (PPOmodules.py:114-125,
    312-332): acceptor and core-chooser action (1 B) + log-prob (4 B) per unit, and with free prices the price
    chooser's state (4 B), action (1 B), log-prob (4 B) and the env's price action (1 B) per offer unit. A fused
    env + act launch (k_env_rollout_act_free) writes these beside the round's bytes and reads no observation
    back: its roofline counts env_round_bytes + these."""
    N, C, L = shape.n_agents, shape.n_cores, shape.collection_length
    return 5 * N * C + 5 * N * L + (10 * N * L if free else 0)


def cpu_baseline(seconds_budget: float = 20.0):
    """The CPU restatement timed on this host: oracle env step (C, OpenMP) + torch-CPU
    policy act / PPO update of the same cfg3 loop, on a bounded sample of replicas."""
    import numpy as np
    import torch

    from oracle import pyoracle
    from oracle.ppo_ref import RefActorCritic

    # the box's CPU share is OMP_NUM_THREADS (os.sched_getaffinity shows the whole machine)
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "0") or 10**6))
    torch.set_num_threads(cores)
    cfg = pyoracle.abi.named_config("cfg3")
    s = pyoracle.abi.config_shape(cfg)
    N, C, L = s["N"], s["C"], s["L"]
    E, T = 64, 200
    batch = pyoracle.OracleBatch(cfg, E, seed=1)
    torch.manual_seed(0)
    nets = dict(acc=[RefActorCritic(s["acc_obs_dim"], s["acc_actions"]) for _ in range(N)],
                off=[RefActorCritic(s["off_obs_dim"], s["off_actions"]) for _ in range(N)],
                price=[RefActorCritic(4, s["price_actions"]) for _ in range(N)])
    opt = {k: [torch.optim.Adam([{"params": n.actor.parameters(), "lr": 3e-3},
                                 {"params": n.critic.parameters(), "lr": 1e-2}]) for n in v] for k, v in nets.items()}
    acc_obs = np.zeros((E, N, C, s["acc_obs_stride"]), np.int8)
    off_obs = np.zeros((E, N, L, s["off_obs_stride"]), np.int8)
    buf = dict(acc=[], off=[], price=[])

    def act(group, x):  # x [E, N, U, D] float -> actions [E, N, U]
        out = torch.empty(x.shape[:3], dtype=torch.long)
        lps = torch.empty(x.shape[:3])
        with torch.no_grad():
            for a in range(N):
                probs = group[a].actor(x[:, a])
                d = torch.distributions.Categorical(probs)
                act_ = d.sample()
                out[:, a], lps[:, a] = act_, d.log_prob(act_)
        return out, lps

    t0 = time.perf_counter()
    rounds = 0
    for t in range(T):
        xa = torch.from_numpy(acc_obs[..., : s["acc_obs_dim"]]).float()
        xo = torch.from_numpy(off_obs[..., : s["off_obs_dim"]]).float()
        ao, lpo = act(nets["off"], xo)
        idx = (2 * ao).unsqueeze(-1) + torch.arange(2)
        pin = torch.cat((torch.gather(xo, 3, idx), xo[..., 2 * C:2 * C + 2]), -1)
        pin = torch.where((ao == 0).unsqueeze(-1), torch.full_like(pin, -5.0), pin)
        ap, lpp = act(nets["price"], pin)
        aa, lpa = act(nets["acc"], xa)
        price = torch.where(ao == 0, torch.full_like(ap, -5), ap)
        res = batch.step(aa.numpy().astype(np.int8), ao.numpy().astype(np.int8), price.numpy().astype(np.int8),
                         threads=cores)
        acc_obs, off_obs = res["acc_obs"], res["off_obs"]
        buf["acc"].append((xa, aa, lpa, torch.from_numpy(res["acceptor"]).float()))
        buf["off"].append((xo, ao, lpo, torch.from_numpy(res["offer"])))
        buf["price"].append((pin, ap, lpp, torch.from_numpy(res["price"])))
        rounds += 1
        if rounds >= 8 and time.perf_counter() - t0 > seconds_budget:
            break
    # one PPO update on 2 sub-units per agent and unit type (locally shared, K = 1)
    for kind, units in (("acc", C), ("off", L), ("price", L)):
        xs = torch.stack([b[0] for b in buf[kind]], 1)        # [E, R, N, U, D]
        as_ = torch.stack([b[1] for b in buf[kind]], 1)
        lp = torch.stack([b[2] for b in buf[kind]], 1)
        rw = torch.stack([b[3] for b in buf[kind]], 1)
        for a in range(N):
            for sub in range(2):
                u = sub % units
                x = xs[:, :, a, u].reshape(-1, xs.shape[-1])
                g = torch.zeros_like(rw[:, :, a, u])
                run = torch.zeros(E)
                for r in range(rw.shape[1] - 1, -1, -1):
                    run = rw[:, r, a, u] + 0.95 * run
                    g[:, r] = run
                g = ((g - g.mean(1, keepdim=True)) / (g.std(1, keepdim=True) + 1e-7)).reshape(-1)
                logp, v, ent = nets[kind][a].evaluate(x, as_[:, :, a, u].reshape(-1))
                ratio = torch.exp(logp - lp[:, :, a, u].reshape(-1))
                adv = g - v.detach()
                loss = (-torch.min(ratio * adv, ratio.clamp(0.8, 1.2) * adv) + 0.5 * ((v - g) ** 2).mean()
                        - 0.01 * ent).mean()
                opt[kind][a].zero_grad()
                loss.backward()
                opt[kind][a].step()
    dt = time.perf_counter() - t0
    return {"value": E * N * rounds / dt, "unit": "agent-env-steps/s", "cores": cores, "kind": "port",
            "sample": "%d replicas x %d rounds of cfg3 (oracle C env step, OpenMP %d threads) + torch-CPU act and "
                      "one locally-shared PPO update (K=1, 2 sub-units per agent and unit type)" % (E, rounds, cores)}


def cpu_baseline_e1(seconds_budget: float = 10.0):
    """BASELINE.md's CPU form 1: one env (E = 1) on one thread, acting the way the reference's loop
    does (trainPPO.py:160-167: every unit's ActorCritic.act on its own 1-row observation,
    PPOmodules.py:53-63), the C oracle's env step, and one locally-shared PPO update (K = 1, 2
    sub-units per agent and unit type) per 200 rounds when the sample reaches them."""
    import numpy as np
    import torch

    from oracle import pyoracle
    from oracle.ppo_ref import RefActorCritic

    torch.set_num_threads(1)
    cfg = pyoracle.abi.named_config("cfg3")
    s = pyoracle.abi.config_shape(cfg)
    N, C, L = s["N"], s["C"], s["L"]
    batch = pyoracle.OracleBatch(cfg, 1, seed=1)
    torch.manual_seed(0)
    nets = dict(acc=[RefActorCritic(s["acc_obs_dim"], s["acc_actions"]) for _ in range(N)],
                off=[RefActorCritic(s["off_obs_dim"], s["off_actions"]) for _ in range(N)],
                price=[RefActorCritic(4, s["price_actions"]) for _ in range(N)])
    acc_obs = np.zeros((1, N, C, s["acc_obs_stride"]), np.int8)
    off_obs = np.zeros((1, N, L, s["off_obs_stride"]), np.int8)

    def act1(net, row):
        with torch.no_grad():
            d = torch.distributions.Categorical(net.actor(torch.from_numpy(row).float()))
            a = d.sample()
            return int(a), float(d.log_prob(a))

    t0 = time.perf_counter()
    rounds = 0
    while rounds < 8 or time.perf_counter() - t0 < seconds_budget:
        aa = np.zeros((1, N, C), np.int8)
        ao = np.zeros((1, N, L), np.int8)
        ap = np.full((1, N, L), -5, np.int8)
        for a in range(N):  # per agent: offer units (core + price chooser), then acceptors (Agent.py:504-515)
            for l in range(L):
                x = off_obs[0, a, l, : s["off_obs_dim"]]
                core, _ = act1(nets["off"][a], x)
                pin = np.full(4, -5, np.int8) if core == 0 else np.concatenate((x[2 * core:2 * core + 2], x[-2:]))
                price, _ = act1(nets["price"][a], pin)
                ao[0, a, l], ap[0, a, l] = core, (-5 if core == 0 else price)
            for c in range(C):
                aa[0, a, c], _ = act1(nets["acc"][a], acc_obs[0, a, c, : s["acc_obs_dim"]])
        res = batch.step(aa, ao, ap, threads=1)
        acc_obs, off_obs = res["acc_obs"], res["off_obs"]
        rounds += 1
    dt = time.perf_counter() - t0
    return {"value": N * rounds / dt, "unit": "agent-env-steps/s", "cores": 1, "kind": "port",
            "sample": "1 replica x %d rounds of cfg3 on one thread: per-unit torch-CPU ActorCritic.act (the "
                      "reference loop's call pattern) + the C oracle's env step; no update in the sample" % rounds}


ROLLOUT_STREAMS = 1   # replica parts on separate HIP streams in the rollout (Trainer rollout_streams)
SAMPLE_EVERY = 8      # rounds between timed env launches


def committed_traffic(alg_bytes_per_launch, variant="", kernel="k_env_step"):
    """HBM bytes per k_env_step launch from the committed PMC passes of this workload
    (profiles/*/traffic.json, written by profiles/run_profile.sh: FETCH_SIZE doubled per the
    gfx950 correction + WRITE_SIZE, per launch): the most recent measurement by its ``measured_at``
    stamp (UTC, written by traffic_from_pmc.py; not by directory name, whose order is not the
    order of the rounds); None if absent."""
    import glob
    best = None
    for p in glob.glob(os.path.join(REPO, "profiles", "*", "traffic.json")):
        try:
            with open(p) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        # the passes of this workload's kernel variant (same algorithmic bytes per launch)
        if (d.get("kernel") == kernel and d.get("bytes") and d.get("algorithmic_bytes") == alg_bytes_per_launch
                and d.get("variant", "") == variant):
            key = (d.get("measured_at", ""), p)
            if best is None or key > best[0]:
                best = (key, {"bytes": d["bytes"], "source": os.path.relpath(p, REPO),
                              "measured_at": d.get("measured_at"), "vs_algorithmic": d["bytes"] / alg_bytes_per_launch})
    return best[1] if best else None


OTHER = {  # BASELINE configs[1], [3], [4]: per-GPU replicas of the 1-GPU / 8-GPU sharded workloads
    "cfg2": dict(envs=4096, what="4096 env replicas x 4 agents x 4 cores, fixPrices, PPO globallySharedParameters"),
    "cfg4": dict(envs=8192, what="16 agents x 16 cores x 3 slots, freePrices, divided PPO (the aggregated acceptor's "
                                 "(O+1)^C actions are infeasible, DESIGN.md), 65536 replicas / 8 GPUs = 8192 per GPU"),
    "cfg5": dict(envs=8192, what="32 agents x 32 cores x 3 slots, freePrices, Branching DQN on compact observations, "
                                 "65536 replicas / 8 GPUs = 8192 per GPU"),
}


def bench_other(args):
    """The other BASELINE workloads on this rank (informational lines; the headline is cfg3):
    cfg2 / cfg4 = PPO iterations of the batched trainer; cfg5 = Branching DQN frames (one step =
    --update-step frames: act, env step, replay, one update per role per frame)."""
    import torch
    import torch.distributed as dist

    world, rank, local_rank = init_ranks(args)
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    importlib.import_module("marl-scheduling_amd")
    spec = OTHER[args.config]
    E = args.envs or spec["envs"]
    T = args.update_step
    if args.config == "cfg5":
        bdqn = importlib.import_module("marl-scheduling_amd.bdqn")
        abi = importlib.import_module("marl-scheduling_amd.abi")
        tr = bdqn.BDQNTrainer(abi.named_config("cfg5"), n_envs=E, bcfg=bdqn.BDQNConfig(memory_frames=64,
                                                                                      learning_starts=8),
                              seed=rank, device=device)
        run = lambda: [tr.step() for _ in range(T)]
        N = tr.N
    else:
        trainer_mod = importlib.import_module("marl-scheduling_amd.trainer")
        tr = trainer_mod.Trainer.from_named(args.config, n_envs=E, update_step=T, seed=0, device=device, rank=rank,
                                            world_size=world)
        tr.record_launch_spans(SAMPLE_EVERY)
        tr.use_graph = not args.no_graph
        run = tr.iteration
        N = tr.N
    for _ in range(max(args.warmup, 1)):
        run()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    if hasattr(tr, "timings"):
        tr.timings = dict(rollout=0.0, update=0.0)
    # every timed iteration's env launch spans (a device copy after it), as in main()
    span_hist = None
    if args.config != "cfg5":
        sampled = tr.sampled_spans()
        span_hist = torch.zeros((args.steps,) + tuple(sampled.shape), dtype=sampled.dtype, device=device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        run()
        if span_hist is not None:
            span_hist[i].copy_(sampled)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if tr.flags():
        raise SystemExit("env error flags set: 0x%x" % tr.flags())
    value = world * E * N * T * args.steps / elapsed
    result = {"metric": "agent-env-steps/sec (whole node), %s" % args.config, "value": value,
              "unit": "agent-env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
              "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
              "vs_baseline": None, "dtype": "int8/f32", "data": "synthetic (reference spawn sampler, random-init nets)",
              "config": {"workload": "%s: %s; one step = %d rounds%s" % (args.config, spec["what"], T,
                                                                       " + update" if args.config != "cfg5" else ""),
                         "replicas_per_gpu": E, "rounds_per_step": T,
                         "world_size": dist.get_world_size() if world > 1 else 1,
                         "replicas_total": E * world}}
    tm = dict(tr.timings)
    result["breakdown_ms_per_step"] = {k: v / args.steps * 1e3 for k, v in tm.items()}
    if args.config == "cfg5":
        result["roofline"] = bdqn_act_roofline(tr, device)
    else:
        per_iter_us = [tr.launch_spans_us(span_hist[i]) for i in range(args.steps)]
        launch_us = [v for it in per_iter_us for v in it]
        b_round = env_round_bytes(tr.env.shape, tr.cfg.new_jobs_per_round, tr.free, tr.compact)
        result["roofline"] = env_roofline(b_round, E, launch_us, tr.compact)
        result["roofline"]["avg_launch_us_per_iteration"] = [sum(v) / len(v) for v in per_iter_us]
        result["roofline"]["clock_mhz"] = median_clock(tr, span_hist)
        if getattr(tr, "fused_step", False):  # cfg2: the env launch also samples the next round's actions
            whole = getattr(tr, "fused_rollout", False)
            result["roofline"]["kernel"] = "ms::k_env_rollout_act" if whole else "ms::k_env_step_act"
            result["roofline"]["fused_next_act"] = (
                "each round also holds round t+1's acting (offer + acceptor units from the observations in its "
                "LDS); bytes are the env round's alone" +
                ("; one launch runs all %d rounds: avg_launch_us = its span / %d" % (tr.T, tr.T) if whole else ""))
        result["act_roofline"] = act_roofline(tr, device)
        if getattr(tr, "fused_step", False):
            result["act_roofline"]["rollout_use"] = "round 0 only; rounds 1..T-1 act inside the env launch"
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense f32 matrix (v_mfma_f32_16x16x4_f32) peak
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 matrix peak (no sparsity)


def bdqn_act_roofline(tr, device, reps: int = 10):
    """The acceptor role's fused act kernel (k_bdqn_act<7>): algorithmic flops per launch
    = 2 x rows x (128*128 + 128 + 128 * ac_dim * n) (trunk, value head, advantage heads) over its
    average duration between HIP events on its stream. The trunk and heads run on the bf16 MFMA with
    both operands as three exact bf16 terms, six bf16 products per f32 product: the peak of that
    method is the dense bf16 peak / 6, and `mfma_issued` is the bf16 rate the kernel sustains."""
    import torch

    actor = tr.actors["acc"]
    q = actor.q
    rows = tr.E * tr.N
    slot = tr.head  # the frame the next act reads
    h1 = actor.layer1_compact(tr.core_rows[slot], tr.core_owner[slot], tr.N)
    st = torch.cuda.current_stream(device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    actor.act(h1=h1)
    ev[0].record(st)
    for _ in range(reps):
        actor.act(h1=h1)
    ev[1].record(st)
    ev[1].synchronize()
    sec = ev[0].elapsed_time(ev[1]) / 1e3 / reps
    flops = 2.0 * rows * (128 * 128 + 128 + 128 * q.ac_dim * q.n)
    achieved = flops / sec / 1e12
    peak = BF16_MFMA_PEAK_TFLOPS / 6
    return {"kernel": "ms::k_bdqn_act<7, false>", "bound": "mfma", "achieved": achieved,
            "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
            "method": "three-term bf16 operands, 6 bf16 MFMA products per f32 product (peak = bf16 dense / 6)",
            "mfma_issued": {"achieved": 6 * achieved, "peak": BF16_MFMA_PEAK_TFLOPS,
                            "frac": 6 * achieved / BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s"},
            "f32_mfma_peak": F32_MFMA_PEAK_TFLOPS,
            "flops_per_launch": flops, "avg_launch_us": sec * 1e6, "rows_per_launch": rows,
            "launch_timing": "HIP events around %d launches on the current frame's h1, after the timed region" % reps}


def act_roofline(tr, device, reps: int = 20):
    """One round's acting launch(es) of the PPO trainer (replica part 0: k_act_pair at cfg3) timed
    with HIP events around graph replays of `reps` repeats of round 0, after the timed region.
    Algorithmic flops = 2 (D*16 + 16*16 + 16*A) per row that runs through the MFMA tiles: every
    offer (core chooser) row and, with compact acceptor rows, one owner row per core (the foreign
    rows are sampled from the group's common row; the price chooser from its table), against the
    dense f32 MFMA peak. The kernel is VALU-issue bound (softmax, sampling, input packing), so the
    fraction says how much of the matrix peak acting reaches, not what bounds it."""
    import torch

    e0, e1 = tr.env.parts[0][1], tr.env.parts[0][2]
    E, N, C, L = e1 - e0, tr.N, tr.C, tr.L
    # round 0's act, `reps` times in one HIP graph (as the rollout replays it: eager launches from
    # Python would time the host), on a stream of its own
    st = torch.cuda.Stream(device)
    saved = tr.streams[0]
    tr.streams[0] = st
    try:
        with torch.cuda.stream(st):
            tr._act_part(0, 0)  # warm
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with importlib.import_module("marl-scheduling_amd._lib").hip_capture(g, stream=st):
            for _ in range(reps):
                tr._act_part(0, 0)
    finally:
        tr.streams[0] = saved
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    with torch.cuda.stream(st):
        g.replay()
        ev[0].record(st)
        for _ in range(5):
            g.replay()
        ev[1].record(st)
    ev[1].synchronize()
    sec = ev[0].elapsed_time(ev[1]) / 1e3 / (5 * reps)
    fl = lambda g: 2.0 * (g.D * g.H + g.H * g.H + g.H * g.A)
    off = tr.off.group.policy_old
    acc = tr.acc.group.policy_old
    off_rows = E * N * L
    acc_rows = E * C if tr.compact else E * N * C
    flops = fl(off) * off_rows + fl(acc) * acc_rows
    ref_flops = fl(off) * off_rows + fl(acc) * E * N * C
    if tr.free:
        ref_flops += fl(tr.price.group.policy_old) * off_rows
    achieved = flops / sec / 1e12
    kern = ("ms::k_act_pair (offer + price table + compact acceptors, one launch)" if tr.compact and tr.free
            else "ms::k_act (offers) + ms::k_act / k_act_common (acceptors)")
    return {"kernel": kern, "bound": "mfma",
            "achieved": achieved, "peak": F32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / F32_MFMA_PEAK_TFLOPS, "traffic": None, "flops_per_launch": flops,
            "mfma_rows": {"offer": off_rows, "acceptor": acc_rows},
            "reference_flops_per_launch": ref_flops, "avg_launch_us": sec * 1e6,
            "launch_timing": "HIP events around 5 replays of a HIP graph of %d repeats of round 0's act, "
                             "after the timed region" % reps}


def median_clock(tr, span_hist):
    """The env waves' median shader clock (MHz) over the timed iterations' recorded launches."""
    v = [c for c in (tr.launch_clock_mhz(h) for h in span_hist) if c is not None]
    return float(np.median(v)) if v else None


def env_roofline(b_round: int, envs: int, launch_us, compact: bool, variant_traffic: bool = True):
    """k_env_step's roofline entry: SURVEY 8(d) algorithmic bytes per env-round x replicas per launch
    over the in-region launch spans (tr.record_launch_spans), averaged over the timed iterations."""
    avg_s = sum(launch_us) / len(launch_us) / 1e6
    achieved = b_round * envs / avg_s / 1e9
    traffic = committed_traffic(b_round * envs, "compact" if compact else "") if variant_traffic else None
    return {"kernel": "ms::k_env_step", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic["bytes"] if traffic else None,
            "traffic_source": traffic["source"] if traffic else None, "variant": "compact" if compact else "",
            "bytes_per_env_round": b_round,
            "envs_per_launch": envs, "avg_launch_us": avg_s * 1e6, "launches_timed": len(launch_us)}


def launch_ranks(n: int, argv) -> int:
    """``--gpus N`` without a torch.distributed launcher: start N rank processes of this script,
    one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), the way
    ``torch.distributed.run --nproc-per-node N`` would. Called before anything touches the GPU
    (the parent never initialises HIP); if one rank fails the others are stopped (their exact
    PIDs). Returns the exit code (0 when every rank succeeded)."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:  # a failed rank would leave the others waiting in a collective
                    q.terminate()
        time.sleep(0.05)
    return rc


def init_ranks(args, backend: str = "nccl"):
    """(world, rank, local_rank) from the launcher's environment; joins the process group for
    world > 1 (RCCL over xGMI on GPUs, gloo for the CPU stub) and checks that the group has the
    --gpus ranks it was asked for."""
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit("--gpus %d but the launcher started %d rank(s)" % (args.gpus, world))
    if world > 1:
        if backend == "nccl":
            import torch
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world:
            raise SystemExit("process group has %d ranks, WORLD_SIZE %d" % (dist.get_world_size(), world))
    return world, rank, local_rank


def bench_stub(args):
    """The launcher and process-group path without a GPU (gloo): every rank joins, checks in with
    an all-reduce of ones, and rank 0 prints what the real bench prints about the ranks."""
    import torch
    import torch.distributed as dist

    if os.environ.get("MS_STUB_FAIL_RANK", "-") == os.environ.get("RANK"):  # tests: a rank that dies early
        raise SystemExit(3)
    world, rank, _ = init_ranks(args, backend="gloo")
    E = args.envs or 16384
    seen = torch.ones(1)
    replicas = torch.tensor([float(E)])
    if world > 1:
        dist.all_reduce(seen)
        dist.all_reduce(replicas)
    line = {"metric": "launcher stub", "n_gpus": world, "pg_world_size": dist.get_world_size() if world > 1 else 1,
            "ranks_reported": int(seen.item()), "replicas_per_gpu": E, "replicas_total": int(replicas.item()),
            "rank_pids": None}
    if world > 1:
        pids = [None] * world
        dist.all_gather_object(pids, os.getpid())
        line["rank_pids"] = pids
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


STEP_SEEDS = (0, 1, 2)
STEP_RING = 200          # rounds of pre-sampled actions, cycled
STEP_WARMUP_ROUNDS = 200
STEP_TIMED_ROUNDS = 2000


def step_kernel_line(E: int, device, world: int, rank: int):
    """the env step kernel alone, actions pre-sampled uniformly into a device ring
    (acceptor [0, A_acc), core chooser [0, A_off), price [0, A_pc), price -5 where the core action is
    0 as FreePriceOfferPPO sends it), outputs written as the trainer's rollout gets them (compact
    acceptor rows + owners, offer rows, rewards). Per seed: 200 warm-up rounds, then 2000 timed
    rounds (10 replays of a 200-round HIP graph) between HIP events on the launch stream."""
    import torch
    import torch.distributed as dist

    ms = importlib.import_module("marl-scheduling_amd")
    trainer_mod = importlib.import_module("marl-scheduling_amd.trainer")
    cfg = ms.abi.named_config("cfg3")
    s = ms.abi.config_shape(cfg)
    N, C, L = s["N"], s["C"], s["L"]
    per_seed = {}
    for seed in STEP_SEEDS:
        env = ms.BatchedEnv(cfg, E, seed=trainer_mod.env_seed(seed, rank, E), device=device)
        g = torch.Generator(device=device).manual_seed(seed * 7919 + rank)
        ri = lambda hi, shape: torch.randint(0, hi, shape, generator=g, device=device, dtype=torch.int8)
        acc = ri(s["acc_actions"], (STEP_RING, E, N, C))
        off = ri(s["off_actions"], (STEP_RING, E, N, L))
        price = torch.where(off == 0, torch.full_like(off, -5), ri(s["price_actions"], (STEP_RING, E, N, L)))
        obs = env.compact_obs_buffers()
        rew = env.reward_buffers()
        env.reset(obs)
        # every 10th round's launch span (first wave start -> last wave end) and its waves' shader
        # clock, as the main line records them inside the rollout: the two lines compare on one box
        spans = torch.zeros((STEP_RING // 10, E, 4), dtype=torch.int64, device=device)  # >= the launch's waves

        def body():
            for t in range(STEP_RING):
                ev = dict(launch_span=spans[t // 10]) if t % 10 == 0 else None
                env.step(acc[t], off[t], price[t], obs=obs, rewards=rew, events=ev)

        for _ in range(STEP_WARMUP_ROUNDS // STEP_RING):
            body()
        torch.cuda.synchronize(device)
        graph = torch.cuda.CUDAGraph()
        with importlib.import_module("marl-scheduling_amd._lib").hip_capture(graph):
            body()
        stream = torch.cuda.current_stream(device)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        ev[0].record(stream)
        for _ in range(STEP_TIMED_ROUNDS // STEP_RING):
            graph.replay()
        ev[1].record(stream)
        ev[1].synchronize()
        sec = ev[0].elapsed_time(ev[1]) / 1e3
        if world > 1:
            t = torch.tensor([sec], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            sec = float(t.item())
        if env.flags():
            raise SystemExit("env error flags set in the step-kernel run: 0x%x" % env.flags())
        b_round = env_round_bytes(env.shape, cfg.new_jobs_per_round, True, True)
        us = sec / STEP_TIMED_ROUNDS * 1e6
        sp = spans.cpu().numpy()
        span_us, clk = [], []
        for w in sp:
            w = w[w[:, 1] > 0]
            if len(w):
                span_us.append(float(w[:, 1].max() - w[:, 0].min()) / 100.0)
                ok = (w[:, 1] > w[:, 0]) & (w[:, 3] > w[:, 2])
                clk.extend(((w[ok, 3] - w[ok, 2]) / (w[ok, 1] - w[ok, 0]) * 100.0).tolist())
        per_seed[str(seed)] = {"value": world * E * N * STEP_TIMED_ROUNDS / sec, "us_per_round": us,
                               "frac": b_round * E / (us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                               "launch_span_us": sum(span_us) / len(span_us) if span_us else None,
                               "clock_mhz": float(np.median(clk)) if clk else None}
        del graph, env
    vals = [v["value"] for v in per_seed.values()]
    return {"metric": "agent-env-steps/s, env step kernel alone (SURVEY 8(d)(i))", "unit": "agent-env-steps/s",
            "value": sum(vals) / len(vals), "min": min(vals), "max": max(vals), "per_seed": per_seed,
            "seeds": list(STEP_SEEDS), "replicas_per_gpu": E, "n_gpus": world, "warmup_rounds": STEP_WARMUP_ROUNDS,
            "timed_rounds": STEP_TIMED_ROUNDS,
            "actions": "uniform, pre-sampled into a %d-round device ring" % STEP_RING,
            "timing": "HIP events on the launch stream around %d replays of a %d-round HIP graph"
                      % (STEP_TIMED_ROUNDS // STEP_RING, STEP_RING),
            "launch_span": "launch_span_us: first wave start to last wave end of every 10th round's launch "
                           "(the main line's roofline uses the same span inside the rollout); us_per_round also "
                           "holds the gaps between launches"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a launcher's WORLD_SIZE, N > 1 starts N rank processes")
    ap.add_argument("--stub", action="store_true", help="launcher / process-group check on CPU (gloo), no GPU work")
    ap.add_argument("--no-step-kernel", action="store_true", help="skip the env-step-kernel-only line")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--envs", type=int, default=None, help="env replicas per GPU (default: the config's per-GPU share)")
    ap.add_argument("--update-step", type=int, default=200)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager rollout instead of HIP-graph replay")
    ap.add_argument("--rollout-streams", type=int, default=ROLLOUT_STREAMS,
                    help="replica parts stepped on separate HIP streams (env of one part beside act of another)")
    ap.add_argument("--config", default="cfg3", choices=["cfg2", "cfg3", "cfg4", "cfg5"],
                    help="BASELINE config (cfg3 = the headline; cfg2/cfg4/cfg5 are the other BASELINE workloads)")
    args = ap.parse_args()
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))  # nothing has touched the GPU in this process
    if args.stub:
        return bench_stub(args)
    if args.config != "cfg3":
        return bench_other(args)

    import torch
    import torch.distributed as dist

    world, rank, local_rank = init_ranks(args)
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    ms = importlib.import_module("marl-scheduling_amd")
    trainer_mod = importlib.import_module("marl-scheduling_amd.trainer")
    args.envs = args.envs or 16384
    tr = trainer_mod.Trainer.from_named("cfg3", n_envs=args.envs, update_step=args.update_step, seed=0,
                                        device=device, rank=rank, world_size=world,
                                        rollout_streams=args.rollout_streams)
    shape = tr.env.shape

    # Per-launch duration of k_env_step inside the timed region: every SAMPLE_EVERY-th round's env
    # launches record their span (first wave start -> last wave end, s_memrealtime at 100 MHz, two
    # atomics per wave) into a device buffer that the captured rollout graph re-initialises on every
    # replay; the last timed iteration's spans are read after the timed region. (HIP timing events
    # cannot be captured into the graph on ROCm 7.2, neither torch's Event.record nor
    # hipEventRecordWithFlags(hipEventRecordExternal): tools/graph_event_probe.py.)
    tr.record_launch_spans(SAMPLE_EVERY)

    tr.use_graph = not args.no_graph
    for _ in range(max(args.warmup, 1 if tr.use_graph else 0)):
        tr.iteration()  # the first rollout also captures the HIP graph
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    tr.timings = dict(rollout=0.0, update=0.0)
    # every timed iteration's recorded spans, copied on the device after it (~5 MB, a few us): the
    # policy changes as it trains and with it the env's work per round (more executions, spawns), so the
    # span is averaged over all timed iterations, not read from the last one alone
    sampled = tr.sampled_spans()  # the recorded rounds only (~5 MB at cfg3: a few us per copy)
    span_hist = torch.zeros((args.steps,) + tuple(sampled.shape), dtype=sampled.dtype, device=device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        tr.iteration()
        span_hist[i].copy_(sampled)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    timings = dict(tr.timings)
    per_iter_us = [tr.launch_spans_us(span_hist[i]) for i in range(args.steps)]
    launch_us = [v for it in per_iter_us for v in it]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    flags = tr.flags()
    if flags:
        raise SystemExit("env error flags set: 0x%x" % flags)

    rounds = args.update_step * args.steps
    agent_steps = world * args.envs * shape.n_agents * rounds
    value = agent_steps / elapsed
    avg_step_s = sum(launch_us) / len(launch_us) / 1e6
    part_envs = args.envs // args.rollout_streams
    b_env = env_round_bytes(shape, tr.cfg.new_jobs_per_round, tr.free, tr.compact)
    # the one-launch rollout (k_env_rollout_act_free, the default): one launch steps and acts for T rounds; its
    # per-round span covers the env round and the next round's acting, so its bytes add the acting's outputs
    fused = bool(getattr(tr, "fused_rollout_free", False))
    kname = "k_env_rollout_act_free" if fused else "k_env_step"
    b_act = act_out_bytes(shape, tr.free) if fused else 0
    b_round = b_env + b_act
    achieved = b_round * part_envs / avg_step_s / 1e9
    traffic = committed_traffic(b_round * part_envs, "compact" if tr.compact else "", kname)
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "agent-env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8/f32",
        "data": "synthetic (env job stream from the reference spawn sampler, random-init nets)",
        "config": {
            "workload": "cfg3: %d env replicas/GPU x 8 agents x 8 cores, collectionLength 3, freePrices + "
                        "commercialFreePriceReward, PPO locallySharedParameters, UPDATE_STEP %d; one step = one PPO "
                        "iteration (%d rounds + update)" % (args.envs, args.update_step, args.update_step),
            "replicas_per_gpu": args.envs,
            "rounds_per_step": args.update_step,
            "parallelism": "replicas sharded over %d rank(s), RCCL grad all-reduce" % world,
            "world_size": dist.get_world_size() if world > 1 else 1,
            "replicas_total": world * args.envs,
        },
        "roofline": {
            "kernel": "ms::" + kname,
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic["bytes"] if traffic else None,
            "traffic_source": traffic["source"] if traffic else None,
            "bytes_per_env_round": b_round,
            "env_bytes_per_env_round": b_env,
            "act_bytes_per_env_round": b_act,
            "bytes_definition": "SURVEY.md 8(d) judge figure: state r+w, actions, observations delivered (1 B per "
                                "element), rewards; liability entries left out (lower bound)" +
                                ("; + the fused acting's outputs (bench.act_out_bytes: actions, log-probs, price "
                                 "states written per unit)" if fused else ""),
            "acceptor_observations": "compact (owner row per core + owners)" if tr.compact else "materialised",
            "envs_per_launch": part_envs,
            "avg_launch_us": avg_step_s * 1e6,
            "launches_timed": len(launch_us),
            # per timed iteration: the policy trains, so the env's work per round drifts (from random init,
            # the span grows over the first ~20 iterations: profiles/r5q)
            "avg_launch_us_per_iteration": [sum(v) / len(v) for v in per_iter_us],
            # the env waves' shader clock over the same launches (s_memtime cycles / s_memrealtime ticks)
            "clock_mhz": median_clock(tr, span_hist),
            "launch_timing": ("first-wave-start to last-wave-end span (s_memrealtime, 100 MHz) of the one rollout "
                              "launch of every timed iteration (graph replay) / its %d rounds: the env round + "
                              "the next round's acting, per round" % tr.T) if fused else
                             ("first-wave-start to last-wave-end span (s_memrealtime, 100 MHz) of every %d-th "
                              "round's env launches in every timed iteration (graph replay), averaged" % SAMPLE_EVERY),
        },
        "breakdown_ms_per_step": {
            "rollout": timings["rollout"] / args.steps * 1e3,
            "update": timings["update"] / args.steps * 1e3,
            "rollout_mode": ("hip-graph replay" if not args.no_graph else "eager")
                            + (", %d streams" % args.rollout_streams if args.rollout_streams > 1 else ""),
        },
    }
    result["act_roofline"] = act_roofline(tr, device)
    if fused:
        result["act_roofline"]["rollout_use"] = ("round 0 only; rounds 1..T-1 act inside the rollout launch "
                                                 "(k_env_rollout_act_free, one wave per agent)")
    if not args.no_step_kernel:
        del tr  # the trainer's rings are not needed by the step-kernel run
        torch.cuda.empty_cache()
        result["step_kernel"] = step_kernel_line(args.envs, device, world, rank)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline()
        except Exception as exc:  # reported, never fatal for the GPU number
            result["cpu_baseline"] = {"error": repr(exc)}
        try:
            result["cpu_baseline_e1"] = cpu_baseline_e1()
        except Exception as exc:
            result["cpu_baseline_e1"] = {"error": repr(exc)}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
