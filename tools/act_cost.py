"""Kernel-time split of one cfg3 round's acting (offer core chooser alone vs core + price chooser vs
the paired launch with the acceptors), from HIP events around repeated launches."""
import importlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
tr_mod = importlib.import_module("marl-scheduling_amd.trainer")
ppo = importlib.import_module("marl-scheduling_amd.ppo")
tr = tr_mod.Trainer.from_named("cfg3", n_envs=int(os.environ.get("E", 16384)), update_step=8, seed=1, device="cuda:0")
tr.iteration()
t = 3
N, C, L = tr.N, tr.C, tr.L
off_obs = tr.off_obs[t]
out = dict(core_action=tr.off.actions[t], core_logprob=tr.off.logprobs[t], price_state=tr.price_obs[t],
           price_action=tr.price.actions[t], price_logprob=tr.price.logprobs[t], env_price=tr.env_price)
pus = 0
pt = tr.price_table


def timed(fn, n=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n * 1e3


core = tr.off.group.policy_old
price = tr.price.group.policy_old
acc = tr.acc.group.policy_old
res = {
    "core chooser alone (ms_policy_act)": timed(lambda: core.act(off_obs, N * L, 1, 1, action=out["core_action"],
                                                                 logprob=out["core_logprob"])),
    "core + price chooser (ms_offer_act_free)": timed(lambda: ppo.offer_act_free(core, price, off_obs, C, 1, 1, out, price_unit_stride=pus)),
    "acceptors compact (ms_policy_act_compact)": timed(lambda: acc.act_compact(tr.acc_rows[t], tr.acc_owner[t], N * C, 1, 3,
                                                                                tr.acc_common, action=tr.acc.actions[t],
                                                                                logprob=tr.acc.logprobs[t])),
    "paired (ms_act_round_free)": timed(lambda: ppo.act_round_free(core, price, off_obs, acc, tr.acc_rows[t], tr.acc_owner[t],
                                                                   tr.acc_common, C, 1, 1, 3, out, tr.acc.actions[t],
                                                                   tr.acc.logprobs[t], price_unit_stride=pus, price_table=pt)),
    "paired with act fragments (the trainer's launch)": timed(lambda: ppo.act_round_free(
        core, price, off_obs, acc, tr.acc_rows[t], tr.acc_owner[t], tr.acc_common, C, 1, 1, 3, out, tr.acc.actions[t],
        tr.acc.logprobs[t], price_unit_stride=pus, price_table=pt, core_frag=tr.off_frag, acc_frag=tr.acc_frag)),
}
for k, v in res.items():
    print("%-45s %8.2f us" % (k, v))
