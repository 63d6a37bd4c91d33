// capi.cpp — extern "C" boundary of libmarlsched.so (include/marlsched.h).
//
// Host side of the drop-in: validates configurations, owns the device state of
// E env replicas, and enqueues the HIP kernels on the caller's stream.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "ms_layout.h"
#include "ms_dqn.h"
#include "ms_bdqn.h"
#include "ms_wide.h"
#include "ms_ppo.h"

namespace ms {
hipError_t launch_bdqn_update(const BdqnUpd&, hipStream_t);
hipError_t launch_env_init(const Params&, int64_t, uint8_t*, uint32_t*, Liab*, uint64_t, hipStream_t);
hipError_t launch_env_reset(const Params&, int64_t, const uint8_t*, int8_t*, int8_t*, int8_t*, int8_t*, int8_t*,
                            hipStream_t);
hipError_t launch_env_step(const Params&, int64_t, uint8_t*, uint32_t*, Liab*, const StepIO&, hipStream_t);
hipError_t launch_env_step_act(const Params&, int64_t, uint8_t*, uint32_t*, Liab*, const StepIO&, const FusedAct&,
                               hipStream_t);
bool env_step_act_supported(const Params&, int64_t);
hipError_t launch_env_rollout_act(const Params&, int64_t, uint8_t*, uint32_t*, Liab*, const StepIO&, const FusedAct&,
                                  const RoundStride&, int, int, hipStream_t);
hipError_t launch_env_rollout_act_free(const Params&, int64_t, uint8_t*, uint32_t*, Liab*, const StepIO&,
                                       const FusedActFree&, const RoundStrideFree&, int, int, hipStream_t);
bool env_rollout_free_supported(const Params&);
hipError_t launch_env_fill_common(const Params&, int64_t, const StepIO&, const FusedActFree&, const RoundStrideFree&,
                                  int, int, hipStream_t);
hipError_t launch_env_randbelow(const Params&, uint8_t*, uint32_t*, int64_t, uint32_t, uint32_t*, hipStream_t);
hipError_t launch_env_auctioneer(const Params&, int64_t, uint8_t*, uint32_t*, int8_t*, hipStream_t);
hipError_t launch_policy_act(const ms_mlp_params*, const int8_t*, int, int64_t, int, int, const int8_t*, uint64_t,
                             uint64_t, const uint64_t*, const float*, int8_t*, float*, hipStream_t);
hipError_t launch_policy_act_compact(const ms_mlp_params*, const int8_t*, const int8_t*, int, int64_t, int, int, int,
                                     const int8_t*, uint64_t, uint64_t, const uint64_t*, const float*, int8_t*, float*,
                                     hipStream_t);
hipError_t launch_act_round(const ms_mlp_params*, const ms_mlp_params*, const int8_t*, int, int, int,
                            const ms_mlp_params*, const int8_t*, const int8_t*, int, int, int, int, const int8_t*,
                            int64_t, uint64_t, uint64_t, uint64_t, const uint64_t*, int8_t*, float*, int8_t*, int8_t*,
                            float*, int8_t*, int8_t*, float*, const float*, const int16_t*, int, int64_t, hipStream_t);
hipError_t launch_price_table(const ms_mlp_params*, const int8_t*, int, float*, hipStream_t);
size_t act_frag_bytes(const ms_mlp_params*, int);
hipError_t launch_act_prepare(const ms_mlp_params*, const int8_t*, int, void*, hipStream_t);
hipError_t launch_offer_act_free(const ms_mlp_params*, const ms_mlp_params*, const int8_t*, int, int64_t, int, int, int,
                                 uint64_t, uint64_t, const uint64_t*, const float*, int8_t*, float*, int8_t*, int8_t*,
                                 float*, int8_t*, int64_t, hipStream_t);
hipError_t launch_returns(const float*, int, int64_t, int64_t, double, float*, hipStream_t);
hipError_t launch_unit_returns(const void*, int, int, int64_t, int, const int32_t*, int, double, float*, hipStream_t);
hipError_t launch_ppo_grad(const PpoArgs&, const GradOut&, hipStream_t);
int ppo_param_count(int D, int A);
int ppo_partial_rows(int n_chunks, bool keyed);
hipError_t launch_aggregate_obs(const AggArgs&, hipStream_t);
hipError_t launch_decode_aggregated(const int32_t*, long long, int, int, int, int, int8_t*, int8_t*, int*, hipStream_t);
hipError_t launch_adam(const AdamTensor*, int, const double*, int, int64_t, double, double, double, const int64_t*,
                       hipStream_t);
hipError_t launch_dqn_act(const DqnActArgs&, hipStream_t);
hipError_t launch_regen_agent_rows(const RegenArgs&, hipStream_t);
hipError_t launch_dqn_grad(const DqnGradArgs&, const DqnReduceArgs&, hipStream_t);
hipError_t launch_bdqn_w1split(const float*, int, int, int, uint16_t*, hipStream_t);
hipError_t launch_bdqn_l1_base(const float*, const float*, int, int, float*, float*, hipStream_t);
hipError_t launch_bdqn_l1_compact(const BdqnL1Compact&, hipStream_t);
hipError_t launch_bdqn_act(const BdqnAct&, hipStream_t);
hipError_t launch_wide_act(const WideAct&, hipStream_t);
hipError_t launch_wide_grad(const WideRows&, const WideGrads&, const WideReduce&, hipStream_t);
}  // namespace ms

// work split of k_ppo_grad: ~kGradWaves wave chunks over all groups (4 per block), >= 8 tiles of 16 rows each
#ifndef MS_GRAD_WAVES
#define MS_GRAD_WAVES 8192
#endif
static void ppo_split(int64_t rows, int G, int* chunk_tiles, int* n_chunks) {
    constexpr int64_t kGradWaves = MS_GRAD_WAVES;
    int64_t tiles = (rows + 15) / 16;
    int64_t ct = (tiles * G + kGradWaves - 1) / kGradWaves;
    if (ct < 8) ct = 8;
    ct = (ct + 1) & ~1LL;  // whole tile pairs (the dW1 step runs on 32 rows)
    *chunk_tiles = (int)ct;
    int64_t nc = (tiles + ct - 1) / ct;
    *n_chunks = (int)((nc + 3) / 4 * 4);
}

struct ms_env {
    ms_config cfg;
    ms::Params P;
    int64_t E;
    int device;
    uint8_t* recs;
    uint32_t* mt;
    ms::Liab* liab;
    uint32_t* scratch_u32;  // device word for randbelow
    uint32_t* err_host;     // sticky error word in host-coherent memory: set by a round that raised a
                            // fatal per-env flag (ms_layout.h kFatalFlags), read by ms_env_step without a sync
    int64_t round;
};

static thread_local char g_err[512] = "";

static int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) return fail(MS_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

static bool fits_i8(long v) { return v >= -128 && v <= 127; }

static int validate_config(const ms_config* c) {
    if (!c) return fail(MS_EINVAL, "config is NULL");
    if (c->n_agents < 1 || c->n_agents > MS_MAX_AGENTS) return fail(MS_EINVAL, "n_agents must be in [1, %d]", MS_MAX_AGENTS);
    if (c->n_cores < 1 || c->n_cores > MS_MAX_CORES) return fail(MS_EINVAL, "n_cores must be in [1, %d]", MS_MAX_CORES);
    if (c->collection_length < 1 || c->collection_length > MS_MAX_COLLECTION)
        return fail(MS_EINVAL, "collection_length must be in [1, %d]", MS_MAX_COLLECTION);
    if (c->n_agents * c->collection_length > MS_MAX_OFFERS)
        return fail(MS_EINVAL, "n_agents * collection_length must be <= %d", MS_MAX_OFFERS);
    if (c->n_kinds < 1 || c->n_kinds > MS_MAX_KINDS) return fail(MS_EINVAL, "n_kinds must be in [1, %d]", MS_MAX_KINDS);
    for (int i = 0; i < c->n_kinds; i++) {
        if (c->job_priority[i] < 0 || c->job_priority[i] > 127) return fail(MS_EINVAL, "job priorities must be in [0, 127]");
        if (c->job_length[i] < 1 || c->job_length[i] > 127) return fail(MS_EINVAL, "job lengths must be in [1, 127]");
        if (i > 0 && !(c->acc_probability[i] >= c->acc_probability[i - 1]))
            return fail(MS_EINVAL, "accumulated probabilities must be non-decreasing");
    }
    if (!c->free_prices) {
        if (c->n_fix_prices < c->n_kinds) return fail(MS_EINVAL, "fixed prices need one price per job kind");
        for (int i = 0; i < c->n_fix_prices && i < MS_MAX_KINDS; i++)
            if (!fits_i8(c->fix_price[i])) return fail(MS_EINVAL, "fixed prices must fit int8");
    }
    if (c->new_jobs_per_round < 0 || c->new_jobs_per_round > c->collection_length)
        return fail(MS_EINVAL, "new_jobs_per_round must be in [0, collection_length]");
    if (c->n_agents * (c->new_jobs_per_round > 0 ? c->new_jobs_per_round : 1) > 256)
        return fail(MS_EINVAL, "n_agents * new_jobs_per_round must be <= 256");
    long max_rew = (long)c->reward_multiplier * 127;
    if (max_rew > (1L << 24) || max_rew < -(1L << 24)) return fail(MS_EINVAL, "reward_multiplier out of range");
    if (c->episode_length < 1) return fail(MS_EINVAL, "episode_length must be >= 1");
    if (c->liability_cap < 0 || c->liability_cap > 255) return fail(MS_EINVAL, "liability_cap must be in [0, 255]");
    if (c->rng_mode != MS_RNG_CPYTHON_MT19937) return fail(MS_EINVAL, "unknown rng_mode");
    return MS_OK;
}

static int cap_of(const ms_config* c) { return c->liability_cap > 0 ? c->liability_cap : 128; }

extern "C" {

const char* ms_last_error(void) { return g_err; }
int ms_abi_version(void) { return MS_ABI_VERSION; }

int ms_config_shape(const ms_config* cfg, ms_shape* s) {
    int rc = validate_config(cfg);
    if (rc) return rc;
    if (!s) return fail(MS_EINVAL, "shape is NULL");
    ms::Params P = ms::make_params(*cfg, cap_of(cfg));
    memset(s, 0, sizeof(*s));
    s->n_agents = P.N;
    s->n_cores = P.C;
    s->collection_length = P.L;
    s->max_offers = P.O;
    s->acc_obs_dim = P.d_acc;
    s->acc_obs_stride = P.acc_stride;
    s->off_obs_dim = P.d_off;
    s->off_obs_stride = P.off_stride;
    s->acc_actions = P.O + 1;
    s->off_actions = P.C + 1;
    int mp = 0;
    for (int i = 0; i < cfg->n_kinds; i++) mp = cfg->job_priority[i] > mp ? cfg->job_priority[i] : mp;
    s->price_actions = mp + 1;
    s->liability_cap = P.cap;
    s->env_record_bytes = P.rec_bytes;
    return MS_OK;
}

int ms_env_shape(const ms_env* env, ms_shape* out) {
    if (!env) return fail(MS_EINVAL, "env is NULL");
    return ms_config_shape(&env->cfg, out);
}

void ms_env_destroy(ms_env* env) {
    if (!env) return;
    int cur = 0;
    if (hipGetDevice(&cur) == hipSuccess && cur != env->device) (void)hipSetDevice(env->device);
    if (env->recs) (void)hipFree(env->recs);
    if (env->mt) (void)hipFree(env->mt);
    if (env->liab) (void)hipFree(env->liab);
    if (env->scratch_u32) (void)hipFree(env->scratch_u32);
    if (env->err_host) (void)hipHostFree(env->err_host);
    if (cur != env->device) (void)hipSetDevice(cur);
    delete env;
}

int ms_env_create(const ms_config* cfg, int64_t n_envs, uint64_t seed, ms_env** out) {
    if (!out) return fail(MS_EINVAL, "out is NULL");
    *out = nullptr;
    int rc = validate_config(cfg);
    if (rc) return rc;
    if (n_envs < 1 || n_envs > (1LL << 31) - 1) return fail(MS_EINVAL, "n_envs must be in [1, 2^31)");
    ms_env* env = new ms_env();
    env->cfg = *cfg;
    env->P = ms::make_params(*cfg, cap_of(cfg));
    env->E = n_envs;
    env->round = 0;
    HIP_TRY(hipGetDevice(&env->device));
    size_t rec_b = (size_t)n_envs * env->P.rec_bytes;
    size_t mt_b = (size_t)n_envs * 2 * ms::kMtN * sizeof(uint32_t);  // current block + successor
    size_t liab_b = (size_t)n_envs * env->P.C * env->P.cap * sizeof(ms::Liab);
    if (hipMalloc(&env->recs, rec_b) != hipSuccess || hipMalloc(&env->mt, mt_b) != hipSuccess ||
        hipMalloc(&env->liab, liab_b) != hipSuccess || hipMalloc(&env->scratch_u32, 16) != hipSuccess ||
        hipHostMalloc(&env->err_host, 16, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        ms_env_destroy(env);
        return fail(MS_ENOMEM, "device allocation of %zu bytes failed", rec_b + mt_b + liab_b);
    }
    *env->err_host = 0;
    hipError_t e = ms::launch_env_init(env->P, n_envs, env->recs, env->mt, env->liab, seed, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        ms_env_destroy(env);
        return fail(MS_EHIP, "env init: %s", hipGetErrorString(e));
    }
    *out = env;
    return MS_OK;
}

// world.round of replica 0 as stored on the device (authoritative also when the
// steps were replayed from a captured HIP graph); synchronises the device.
int64_t ms_env_round(const ms_env* env) {
    if (!env) return -1;
    int32_t r = -1;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&r, env->recs, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return r;
}

int ms_env_reset(ms_env* env, const ms_obs_out* obs, void* stream) {
    if (!env || !obs) return fail(MS_EINVAL, "env/obs is NULL");
    HIP_TRY(ms::launch_env_reset(env->P, env->E, env->recs, obs->acceptor, obs->offer, obs->auctioneer, obs->core_rows,
                                 obs->core_owner,
                                 (hipStream_t)stream));
    return MS_OK;
}

struct RolloutArgs {
    ms::RoundStride st;
    int n_rounds, act_last;
};
static int env_step_impl(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                         const ms_event_out* ev, const ms::FusedAct* fa, const RolloutArgs* ro, void* stream);
static int fill_io(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                   const ms_event_out* ev, ms::StepIO* out);
static int check_mlp(const ms_mlp_params* p, int32_t obs_stride, int32_t n_units, int32_t units_per_group);

int ms_env_step(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                const ms_event_out* ev, void* stream) {
    return env_step_impl(env, act, obs, rew, ev, nullptr, nullptr, stream);
}

// the checks ms_env_step_act and ms_env_rollout_act share; fills fa
static int fused_act_args(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_event_out* ev,
                          const ms_fused_act* next, const char* who, ms::FusedAct* fa) {
    if (!env || !next) return fail(MS_EINVAL, "env/next is NULL");
    const ms::Params& P = env->P;
    auto bad = [&](const char* why) { return fail(MS_EINVAL, "%s: %s", who, why); };
    if (env->cfg.free_prices) return bad("fixed-price rounds only");
    if (!obs || !obs->core_rows || !obs->core_owner || !obs->offer || obs->acceptor)
        return bad("needs compact acceptor observations (core_rows, core_owner) and offer rows");
    if (!act || !act->acceptor || (ev && ev->metrics)) return bad("the trainer's round only (actions given, no metrics)");
    const ms_mlp_params& o = next->offer;
    const ms_mlp_params& a = next->acceptor;
    if (o.n_groups != 1 || a.n_groups != 1 || o.hidden != 16 || a.hidden != 16 || !o.act_frag || !a.act_frag)
        return bad("one 16-wide net per role with act fragments");
    if (o.in_dim != P.d_off || a.in_dim != P.d_acc || o.n_actions != P.C + 1 || a.n_actions != P.O + 1)
        return bad("net shapes do not match the env");
    if (P.off_stride > 32 || P.acc_stride > 32 || o.n_actions > 16 || a.n_actions > 16 ||
        !ms::env_step_act_supported(P, env->E))
        return bad("shape not supported (one k-step, <= 16 actions, a wave's rows)");
    if (!next->off_action || !next->off_logprob || !next->acc_action || !next->acc_logprob || !next->common_row)
        return bad("NULL output / common row");
    *fa = ms::FusedAct{o, a, next->common_row, next->seed, next->off_offset, next->acc_offset, next->offset_dev,
                       next->off_action, next->off_logprob, next->acc_action, next->acc_logprob};
    return MS_OK;
}

int ms_env_step_act(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                    const ms_event_out* ev, const ms_fused_act* next, void* stream) {
    ms::FusedAct fa;
    const int rc = fused_act_args(env, act, obs, ev, next, "ms_env_step_act", &fa);
    if (rc != MS_OK) return rc;
    return env_step_impl(env, act, obs, rew, ev, &fa, nullptr, stream);
}

int ms_env_rollout_act(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                       const ms_event_out* ev, const ms_fused_act* next, const ms_round_strides* strides,
                       int32_t n_rounds, int32_t act_after_last, void* stream) {
    ms::FusedAct fa;
    const int rc = fused_act_args(env, act, obs, ev, next, "ms_env_rollout_act", &fa);
    if (rc != MS_OK) return rc;
    if (!strides || n_rounds < 1) return fail(MS_EINVAL, "ms_env_rollout_act: strides NULL or n_rounds < 1");
    if (ev && (ev->accepted || ev->terminated))
        return fail(MS_EINVAL, "ms_env_rollout_act: no accepted / terminated event records");
    if (rew && (rew->price || rew->aggregated_offer || rew->aggregated_acceptor))
        return fail(MS_EINVAL, "ms_env_rollout_act: no price / aggregated reward outputs");
    const ms_round_strides& r = *strides;
    RolloutArgs ro{{r.acceptor_action, r.offer_action, r.core_rows, r.core_owner, r.offer_obs, r.offer_reward,
                    r.acceptor_reward, r.agent_reward, r.auctioneer_reward, r.next_off_action, r.next_off_logprob,
                    r.next_acc_action, r.next_acc_logprob, r.offset_step},
                   n_rounds, act_after_last ? 1 : 0};
    return env_step_impl(env, act, obs, rew, ev, &fa, &ro, stream);
}

int ms_env_step_act_supported(const ms_env* env) {
    if (!env) return 0;
    const ms::Params& P = env->P;
    return !env->cfg.free_prices && P.off_stride <= 32 && P.acc_stride <= 32 && P.C + 1 <= 16 && P.O + 1 <= 16 &&
           ms::env_step_act_supported(P, env->E);
}

static int env_step_impl(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                         const ms_event_out* ev, const ms::FusedAct* fa, const RolloutArgs* ro, void* stream) {
    if (!env || !act) return fail(MS_EINVAL, "env/actions is NULL");
    if (!act->acceptor != !act->offer_core)
        return fail(MS_EINVAL, "acceptor and offer_core actions are given together (both NULL: hard-coded agents)");
    if (!act->acceptor && env->cfg.free_prices)
        return fail(MS_EINVAL, "the hard-coded agents are fixed-price only (HardcodedFixPriceEnvironment)");
    if (env->cfg.free_prices && !act->offer_price) return fail(MS_EINVAL, "free prices need offer_price actions");
    // a completed earlier round raised a flag on which the reference raises (assert / TypeError):
    // stop stepping, as the reference would (which replica and flag: ms_env_flags)
    if (__atomic_load_n(env->err_host, __ATOMIC_ACQUIRE))
        return fail(MS_EOVERFLOW, "an earlier round raised a per-env error flag (see ms_env_flags)");
    ms::StepIO io{};
    const int rc = fill_io(env, act, obs, rew, ev, &io);
    if (rc != MS_OK) return rc;
    if (ro)
        HIP_TRY(ms::launch_env_rollout_act(env->P, env->E, env->recs, env->mt, env->liab, io, *fa, ro->st, ro->n_rounds,
                                           ro->act_last, (hipStream_t)stream));
    else if (fa)
        HIP_TRY(ms::launch_env_step_act(env->P, env->E, env->recs, env->mt, env->liab, io, *fa, (hipStream_t)stream));
    else
        HIP_TRY(ms::launch_env_step(env->P, env->E, env->recs, env->mt, env->liab, io, (hipStream_t)stream));
    env->round += ro ? ro->n_rounds : 1;
    return MS_OK;
}

// the launch's StepIO from the caller's structs
static int fill_io(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                   const ms_event_out* ev, ms::StepIO* out) {
    ms::StepIO io{};
    io.err_word = env->err_host;
    io.act_acc = act->acceptor;
    io.act_off = act->offer_core;
    io.act_price = env->cfg.free_prices ? act->offer_price : nullptr;
    io.act_auct = act->auctioneer;
    if (obs) {
        io.obs_acc = obs->acceptor;
        io.obs_off = obs->offer;
        io.obs_auct = obs->auctioneer;
        io.obs_crow = obs->core_rows;
        io.obs_cown = obs->core_owner;
    }
    if (rew) {
        io.rew_offer = rew->offer;
        io.rew_price = rew->price;
        io.rew_acc = rew->acceptor;
        io.rew_auct = rew->auctioneer;
        io.rew_agent = rew->agent;
        io.rew_agg_off = rew->aggregated_offer;
        io.rew_agg_acc = rew->aggregated_acceptor;
    }
    if (ev) {
        io.ev_acc = ev->accepted;
        io.ev_term = ev->terminated;
        io.span = reinterpret_cast<unsigned long long*>(ev->launch_span);
        io.metrics = ev->metrics;
        io.metrics_slots = ev->metrics_slots;
        if (io.metrics && io.metrics_slots < 1) return fail(MS_EINVAL, "ms_env_step: metrics_slots must be >= 1");
    }
    *out = io;
    return MS_OK;
}

static ms::FusedActFree free_act_args(const ms_fused_act_free& n) {
    const ms_price_table* pt = n.price_table;
    return ms::FusedActFree{n.core_chooser, n.price_chooser, n.acceptor, n.common_row,
                            pt ? pt->table : nullptr, pt ? pt->digit : nullptr, pt ? pt->n_keys : 0, n.seed,
                            n.off_offset, n.acc_offset, n.offset_dev, n.core_action, n.core_logprob, n.price_state,
                            n.price_action, n.price_logprob, n.env_price, n.acc_action, n.acc_logprob,
                            n.own_action, n.own_logprob};
}
static ms::RoundStrideFree free_strides(const ms_round_strides_free& r) {
    return ms::RoundStrideFree{r.acceptor_action, r.offer_action, r.core_rows, r.core_owner, r.offer_obs,
                               r.offer_reward, r.price_reward, r.acceptor_reward, r.agent_reward, r.auctioneer_reward,
                               r.next_core_action, r.next_core_logprob, r.next_price_state, r.next_price_action,
                               r.next_price_logprob, r.next_acc_action, r.next_acc_logprob, r.offset_step,
                               r.next_own_action, r.next_own_logprob};
}

int ms_env_rollout_act_free_supported(const ms_env* env) {
    return env && env->cfg.free_prices && ms::env_rollout_free_supported(env->P) ? 1 : 0;
}

int ms_env_rollout_act_free(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                            const ms_event_out* ev, const ms_fused_act_free* next, const ms_round_strides_free* strides,
                            int32_t n_rounds, int32_t act_after_last, void* stream) {
    if (!env || !act || !next || !strides) return fail(MS_EINVAL, "env/act/next/strides is NULL");
    const ms::Params& P = env->P;
    auto bad = [&](const char* why) { return fail(MS_EINVAL, "ms_env_rollout_act_free: %s", why); };
    if (!ms_env_rollout_act_free_supported(env))
        return bad("free prices, N <= 8, max(N, C) <= 16, offer rows <= 32 B / <= 16 core actions, acceptor rows "
                   "33..64 B / 17..32 actions only");
    if (n_rounds < 1) return bad("n_rounds < 1");
    if (!obs || !obs->core_rows || !obs->core_owner || !obs->offer || obs->acceptor || obs->auctioneer)
        return bad("needs compact acceptor observations (core_rows, core_owner) and offer rows only");
    if (!act->acceptor || !act->offer_core || act->offer_price != next->env_price || act->auctioneer)
        return bad("actions: acceptor and offer_core given, offer_price = next->env_price, no auctioneer actions");
    if (ev && (ev->accepted || ev->terminated || ev->metrics)) return bad("no event records or metrics");
    if (rew && (rew->aggregated_offer || rew->aggregated_acceptor)) return bad("no aggregated reward outputs");
    const ms_mlp_params& c = next->core_chooser;
    const ms_mlp_params& p = next->price_chooser;
    const ms_mlp_params& a = next->acceptor;
    const int N = P.N, C = P.C, L = P.L;
    int rc = check_mlp(&c, P.off_stride, N * L, L);
    if (!rc) rc = check_mlp(&p, 4, N * L, L);
    if (!rc) rc = check_mlp(&a, P.acc_stride, N * C, C);
    if (rc) return rc;
    if (c.in_dim != P.d_off || c.n_actions != C + 1 || a.in_dim != P.d_acc || a.n_actions != P.O + 1)
        return bad("net shapes do not match the env");
    if (p.in_dim != 4 || p.n_actions > 16) return bad("price chooser must be 4 -> A with A <= 16");
    if (!c.act_frag || !a.act_frag) return bad("needs act fragments (ms_act_prepare) of both nets");
    const ms_price_table* pt = next->price_table;
    if (!pt || !pt->digit || !pt->table || pt->n_keys < 1 || (int64_t)pt->n_keys * 36 * 4 > 0x7fffffffLL)
        return bad("needs a price table (digit, table, 1 <= n_keys)");
    if (!next->common_row || !next->core_action || !next->core_logprob || !next->price_state || !next->price_action ||
        !next->price_logprob || !next->env_price || !next->acc_action || !next->acc_logprob)
        return bad("NULL output / common row");
    if (!next->own_action != !next->own_logprob) return bad("own_action and own_logprob: both or neither");
    if (env->E * N * L >= (1LL << 24) || env->E * N * C * 4 > 0x7fffffffLL || env->E * N * L * 4 > 0x7fffffffLL ||
        env->E * (int64_t)(N * C) * (N * C) >= (1LL << 32))
        return bad("too many replicas for 32-bit row offsets");
    if (__atomic_load_n(env->err_host, __ATOMIC_ACQUIRE))
        return fail(MS_EOVERFLOW, "an earlier round raised a per-env error flag (see ms_env_flags)");
    ms::StepIO io{};
    rc = fill_io(env, act, obs, rew, ev, &io);
    if (rc != MS_OK) return rc;
    const ms::FusedActFree fa = free_act_args(*next);
    const ms::RoundStrideFree st = free_strides(*strides);
    HIP_TRY(ms::launch_env_rollout_act_free(P, env->E, env->recs, env->mt, env->liab, io, fa, st, n_rounds,
                                            act_after_last ? 1 : 0, (hipStream_t)stream));
    if (!next->defer_common)
        HIP_TRY(ms::launch_env_fill_common(P, env->E, io, fa, st, n_rounds, act_after_last ? 1 : 0, (hipStream_t)stream));
    env->round += n_rounds;
    return MS_OK;
}

int ms_env_rollout_fill_common(const ms_env* env, const ms_obs_out* obs, const ms_fused_act_free* next,
                               const ms_round_strides_free* strides, int32_t n_rounds, int32_t act_after_last,
                               void* stream) {
    if (!env || !obs || !next || !strides) return fail(MS_EINVAL, "env/obs/next/strides is NULL");
    auto bad = [&](const char* why) { return fail(MS_EINVAL, "ms_env_rollout_fill_common: %s", why); };
    if (!ms_env_rollout_act_free_supported(env)) return bad("not an env ms_env_rollout_act_free runs");
    if (n_rounds < 1) return bad("n_rounds < 1");
    if (!obs->core_owner || !next->acceptor.act_frag || !next->acc_action || !next->acc_logprob)
        return bad("needs the owners, the acceptor's act fragments and its outputs");
    if (!next->own_action != !next->own_logprob) return bad("own_action and own_logprob: both or neither");
    if (next->acceptor.n_groups != env->P.N || next->acceptor.n_actions != env->P.O + 1)
        return bad("acceptor net shape does not match the env");
    ms::StepIO io{};
    io.obs_cown = obs->core_owner;
    HIP_TRY(ms::launch_env_fill_common(env->P, env->E, io, free_act_args(*next), free_strides(*strides), n_rounds,
                                       act_after_last ? 1 : 0, (hipStream_t)stream));
    return MS_OK;
}

int ms_env_flags(ms_env* env, uint32_t* flags, void* stream) {
    if (!env || !flags) return fail(MS_EINVAL, "env/flags is NULL");
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    std::vector<uint8_t> h((size_t)env->E * env->P.rec_bytes);
    HIP_TRY(hipMemcpy(h.data(), env->recs, h.size(), hipMemcpyDeviceToHost));
    uint32_t f = 0;
    for (int64_t e = 0; e < env->E; e++) {
        uint32_t v;
        memcpy(&v, h.data() + e * env->P.rec_bytes + 4, 4);
        f |= v;
    }
    *flags = f;
    return MS_OK;
}

int ms_env_randbelow(ms_env* env, int64_t e, uint32_t n, uint32_t* out, void* stream) {
    if (!env || !out) return fail(MS_EINVAL, "env/out is NULL");
    if (e < 0 || e >= env->E) return fail(MS_EINVAL, "env index out of range");
    if (n < 1) return fail(MS_EINVAL, "n must be >= 1");
    HIP_TRY(ms::launch_env_randbelow(env->P, env->recs, env->mt, e, n, env->scratch_u32, (hipStream_t)stream));
    HIP_TRY(hipMemcpyAsync(out, env->scratch_u32, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return MS_OK;
}

int ms_env_auctioneer(ms_env* env, int8_t* actions, void* stream) {
    if (!env || !actions) return fail(MS_EINVAL, "env/actions is NULL");
    HIP_TRY(ms::launch_env_auctioneer(env->P, env->E, env->recs, env->mt, actions, (hipStream_t)stream));
    return MS_OK;
}

// word offset of env e's current MT block (record header word 3 = mt_sel, bit 0 = current half)
static size_t mt_block(int64_t e, int32_t sel) { return ((size_t)e * 2 + (sel & 1)) * ms::kMtN; }

int ms_env_get_rng(ms_env* env, int64_t e, uint32_t* words, int32_t* index, void* stream) {
    if (!env || !words || !index) return fail(MS_EINVAL, "NULL argument");
    if (e < 0 || e >= env->E) return fail(MS_EINVAL, "env index out of range");
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    int32_t hdr[4];
    HIP_TRY(hipMemcpy(hdr, env->recs + e * env->P.rec_bytes, sizeof(hdr), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(words, env->mt + mt_block(e, hdr[3]), 4 * ms::kMtN, hipMemcpyDeviceToHost));
    *index = hdr[2];
    return MS_OK;
}

int ms_env_set_rng(ms_env* env, int64_t e, const uint32_t* words, int32_t index, void* stream) {
    if (!env || !words) return fail(MS_EINVAL, "NULL argument");
    if (e < 0 || e >= env->E) return fail(MS_EINVAL, "env index out of range");
    if (index < 0 || index > ms::kMtN) return fail(MS_EINVAL, "MT index must be in [0, 624]");
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    // current block = half 0; the successor half is recomputed before the env's next draw
    const int32_t hdr[2] = {index, 0};
    HIP_TRY(hipMemcpy(env->mt + mt_block(e, 0), words, 4 * ms::kMtN, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(env->recs + e * env->P.rec_bytes + 8, hdr, sizeof(hdr), hipMemcpyHostToDevice));
    return MS_OK;
}

#define REC_I8(base, off, i) (*(int8_t*)((base) + (off) + (i)))
#define REC_U8(base, off, i) (*(uint8_t*)((base) + (off) + (i)))
#define REC_I32(base, off, i) (*(int32_t*)((base) + (off) + 4 * (i)))

int ms_env_export(ms_env* env, const ms_state_host* o, void* stream) {
    if (!env || !o) return fail(MS_EINVAL, "env/out is NULL");
    const ms::Params& P = env->P;
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    std::vector<uint8_t> rec((size_t)env->E * P.rec_bytes);
    std::vector<uint32_t> mt((size_t)env->E * 2 * ms::kMtN);
    std::vector<ms::Liab> lb((size_t)env->E * P.C * P.cap);
    HIP_TRY(hipMemcpy(rec.data(), env->recs, rec.size(), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(mt.data(), env->mt, mt.size() * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(lb.data(), env->liab, lb.size() * sizeof(ms::Liab), hipMemcpyDeviceToHost));
    const int C = P.C, NL = P.NL, cap = P.cap;
    for (int64_t e = 0; e < env->E; e++) {
        const uint8_t* b = rec.data() + e * P.rec_bytes;
        if (o->round) o->round[e] = REC_I32(b, 0, 0);
        if (o->flags) o->flags[e] = (uint32_t)REC_I32(b, 4, 0);
        if (o->mt_index) o->mt_index[e] = REC_I32(b, 8, 0);
        for (int c = 0; c < C; c++) {
            if (o->core_owner) o->core_owner[e * C + c] = REC_I8(b, P.o_core_owner, c);
            if (o->core_kind) o->core_kind[e * C + c] = REC_I8(b, P.o_core_kind, c);
            if (o->core_rem) o->core_rem[e * C + c] = REC_I8(b, P.o_core_rem, c);
            if (o->core_birth) o->core_birth[e * C + c] = REC_I32(b, P.o_core_birth, c);
            int n = REC_U8(b, P.o_liab_n, c);
            if (o->liab_n) o->liab_n[e * C + c] = n;
            if (o->liab)
                for (int k = 0; k < cap; k++) {
                    int32_t* d = o->liab + (((size_t)e * C + c) * cap + k) * 5;
                    if (k < n) {
                        const ms::Liab& le = lb[((size_t)e * C + c) * cap + k];
                        d[0] = le.offerer;
                        d[1] = le.recipient;
                        d[2] = le.price;
                        d[3] = le.nec;
                        d[4] = le.round;
                    } else {
                        d[0] = d[1] = d[2] = d[3] = d[4] = 0;
                    }
                }
        }
        for (int i = 0; i < NL; i++) {
            size_t j = (size_t)e * NL + i;
            if (o->slot_kind) o->slot_kind[j] = REC_I8(b, P.o_slot_kind, i);
            if (o->slot_rem) o->slot_rem[j] = REC_I8(b, P.o_slot_rem, i);
            if (o->slot_wait) o->slot_wait[j] = REC_I8(b, P.o_slot_wait, i);
            if (o->slot_birth) o->slot_birth[j] = REC_I32(b, P.o_slot_birth, i);
            if (o->offer_core) o->offer_core[j] = REC_I8(b, P.o_offer_core, i);
            if (o->offer_recip) o->offer_recip[j] = REC_I8(b, P.o_offer_recip, i);
            if (o->offer_price) o->offer_price[j] = REC_I8(b, P.o_offer_price, i);
        }
        if (o->mt) memcpy(o->mt + e * ms::kMtN, mt.data() + mt_block(e, REC_I32(b, 12, 0)), ms::kMtN * 4);
    }
    return MS_OK;
}

int ms_env_import(ms_env* env, const ms_state_host* in, void* stream) {
    if (!env || !in) return fail(MS_EINVAL, "env/in is NULL");
    const ms::Params& P = env->P;
    const int N = P.N, C = P.C, L = P.L, NL = P.NL, cap = P.cap;
    std::vector<uint8_t> rec((size_t)env->E * P.rec_bytes, 0);
    std::vector<ms::Liab> lb((size_t)env->E * C * cap);
    memset(lb.data(), 0, lb.size() * sizeof(ms::Liab));
    for (int64_t e = 0; e < env->E; e++) {
        uint8_t* b = rec.data() + e * P.rec_bytes;
        REC_I32(b, 0, 0) = in->round[e];
        REC_I32(b, 4, 0) = in->flags ? (int32_t)in->flags[e] : 0;
        int mti = in->mt_index[e];
        if (mti < 0 || mti > ms::kMtN) return fail(MS_EINVAL, "env %lld: mt_index out of range", (long long)e);
        REC_I32(b, 8, 0) = mti;
        std::vector<int> owned(N + 1, 0), empty(N, 0);
        for (int c = 0; c < C; c++) {
            int k = in->core_kind[e * C + c], own = in->core_owner[e * C + c];
            if (k < -1 || k >= env->cfg.n_kinds) return fail(MS_EINVAL, "env %lld core %d: bad kind", (long long)e, c);
            if (own < 0 || own > N) return fail(MS_EINVAL, "env %lld core %d: bad owner", (long long)e, c);
            if ((k < 0) != (own == 0)) return fail(MS_EINVAL, "env %lld core %d: owner 0 <=> empty job violated", (long long)e, c);
            int rem = in->core_rem[e * C + c];
            if (k >= 0 && (rem < 1 || rem > 127)) return fail(MS_EINVAL, "env %lld core %d: bad remaining length", (long long)e, c);
            REC_I8(b, P.o_core_owner, c) = (int8_t)own;
            REC_I8(b, P.o_core_kind, c) = (int8_t)k;
            REC_I8(b, P.o_core_rem, c) = (int8_t)(k < 0 ? -1 : rem);
            REC_I32(b, P.o_core_birth, c) = k < 0 ? -1 : in->core_birth[e * C + c];
            int n = in->liab_n[e * C + c];
            if (n < 0 || n > cap) return fail(MS_EINVAL, "env %lld core %d: liability chain too long", (long long)e, c);
            REC_U8(b, P.o_liab_n, c) = (uint8_t)n;
            for (int q = 0; q < n; q++) {
                const int32_t* d = in->liab + (((size_t)e * C + c) * cap + q) * 5;
                if (d[0] < 1 || d[0] > N || d[1] < 0 || d[1] > N || !fits_i8(d[2]) || d[3] < 1 || d[3] > 127)
                    return fail(MS_EINVAL, "env %lld core %d: bad liability entry", (long long)e, c);
                ms::Liab& le = lb[((size_t)e * C + c) * cap + q];
                le.offerer = (int8_t)d[0];
                le.recipient = (int8_t)d[1];
                le.price = (int8_t)d[2];
                le.nec = (int8_t)d[3];
                le.round = d[4];
            }
            owned[own]++;
        }
        for (int i = 0; i < NL; i++) {
            size_t j = (size_t)e * NL + i;
            int k = in->slot_kind[j];
            if (k < -1 || k >= env->cfg.n_kinds) return fail(MS_EINVAL, "env %lld slot %d: bad kind", (long long)e, i);
            int rem = in->slot_rem[j];
            if (k >= 0 && (rem < 1 || rem > 127)) return fail(MS_EINVAL, "env %lld slot %d: bad remaining length", (long long)e, i);
            REC_I8(b, P.o_slot_kind, i) = (int8_t)k;
            REC_I8(b, P.o_slot_rem, i) = (int8_t)(k < 0 ? -1 : rem);
            REC_I8(b, P.o_slot_wait, i) = (int8_t)(k < 0 ? 0 : (in->slot_wait[j] != 0));
            REC_I32(b, P.o_slot_birth, i) = k < 0 ? -1 : in->slot_birth[j];
            if (k < 0) empty[i / L]++;
            int oc = in->offer_core[j];
            if (oc >= 0) {
                if (oc >= C || k < 0) return fail(MS_EINVAL, "env %lld slot %d: bad pending offer", (long long)e, i);
                // offers to a core are addressed to its owner (world.py:428 runs after the tick)
                if (in->offer_recip[j] != in->core_owner[e * C + oc])
                    return fail(MS_EINVAL, "env %lld slot %d: offer recipient is not the core owner", (long long)e, i);
                if (!fits_i8(in->offer_price[j])) return fail(MS_EINVAL, "env %lld slot %d: price must fit int8", (long long)e, i);
                REC_I8(b, P.o_offer_core, i) = (int8_t)oc;
                REC_I8(b, P.o_offer_recip, i) = (int8_t)in->offer_recip[j];
                REC_I8(b, P.o_offer_price, i) = (int8_t)in->offer_price[j];
            } else {
                REC_I8(b, P.o_offer_core, i) = -1;
                REC_I8(b, P.o_offer_recip, i) = 0;
                REC_I8(b, P.o_offer_price, i) = 0;
            }
        }
        for (int a = 0; a < N; a++)  // numberOfFreeSlots >= len(ownedCores) (world.py:371-373 keeps it)
            if (empty[a] < owned[a + 1])
                return fail(MS_EINVAL, "env %lld agent %d: fewer free slots than owned cores", (long long)e, a + 1);
    }
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipMemcpy(env->recs, rec.data(), rec.size(), hipMemcpyHostToDevice));
    // current blocks = half 0 (record header mt_sel = 0: successors are recomputed on the device)
    HIP_TRY(hipMemcpy2D(env->mt, 2 * ms::kMtN * 4, in->mt, ms::kMtN * 4, ms::kMtN * 4, (size_t)env->E,
                        hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(env->liab, lb.data(), lb.size() * sizeof(ms::Liab), hipMemcpyHostToDevice));
    env->round = in->round[0];
    *env->err_host = 0;
    for (int64_t e = 0; e < env->E; e++)
        if (in->flags && (in->flags[e] & MS_FATAL_FLAGS)) *env->err_host = 1;
    return MS_OK;
}

static int check_mlp(const ms_mlp_params* p, int32_t obs_stride, int32_t n_units, int32_t units_per_group) {
    if (!p) return fail(MS_EINVAL, "NULL params");
    if (!p->w1 || !p->b1 || !p->w2 || !p->b2 || !p->w3 || !p->b3) return fail(MS_EINVAL, "NULL weight");
    if (p->hidden != 16) return fail(MS_EINVAL, "hidden width %d not built (16 only)", p->hidden);
    if (p->n_actions < 1 || p->n_actions > 127) return fail(MS_EINVAL, "n_actions must be in [1, 127]");
    if (p->in_dim < 1 || p->in_dim > 256 || obs_stride < p->in_dim || obs_stride > 256 || (obs_stride & 3))
        return fail(MS_EINVAL, "bad in_dim / obs stride (<= 256, multiple of 4)");
    if (units_per_group < 1 || p->n_groups < 1 || units_per_group * p->n_groups != n_units)
        return fail(MS_EINVAL, "units_per_group * n_groups must equal n_units");
    return MS_OK;
}

int ms_policy_act(const ms_mlp_params* p, const int8_t* obs, int32_t obs_stride, int64_t n_envs, int32_t n_units,
                  int32_t units_per_group, uint64_t seed, uint64_t offset, const uint64_t* offset_dev,
                  const float* uniforms, int8_t* action, float* logprob, void* stream) {
    if (!obs || !action || !logprob) return fail(MS_EINVAL, "NULL argument");
    int rc = check_mlp(p, obs_stride, n_units, units_per_group);
    if (rc) return rc;
    if (n_envs < 1) return fail(MS_EINVAL, "n_envs must be >= 1");
    HIP_TRY(ms::launch_policy_act(p, obs, obs_stride, n_envs, n_units, units_per_group, nullptr, seed, offset,
                                  offset_dev, uniforms, action, logprob, (hipStream_t)stream));
    return MS_OK;
}

int ms_policy_act_common(const ms_mlp_params* p, const int8_t* obs, int32_t obs_stride, int64_t n_envs,
                         int32_t n_units, int32_t units_per_group, const int8_t* common_row, uint64_t seed,
                         uint64_t offset, const uint64_t* offset_dev, const float* uniforms, int8_t* action,
                         float* logprob, void* stream) {
    if (!obs || !action || !logprob || !common_row) return fail(MS_EINVAL, "NULL argument");
    int rc = check_mlp(p, obs_stride, n_units, units_per_group);
    if (rc) return rc;
    if (n_envs < 1) return fail(MS_EINVAL, "n_envs must be >= 1");
    HIP_TRY(ms::launch_policy_act(p, obs, obs_stride, n_envs, n_units, units_per_group, common_row, seed, offset,
                                  offset_dev, uniforms, action, logprob, (hipStream_t)stream));
    return MS_OK;
}

int ms_policy_act_compact(const ms_mlp_params* p, const int8_t* core_rows, const int8_t* core_owner,
                          int32_t obs_stride, int64_t n_envs, int32_t n_units, int32_t units_per_group, int32_t n_cores,
                          const int8_t* common_row, uint64_t seed, uint64_t offset, const uint64_t* offset_dev,
                          const float* uniforms, int8_t* action, float* logprob, void* stream) {
    if (!core_rows || !core_owner || !action || !logprob || !common_row) return fail(MS_EINVAL, "NULL argument");
    int rc = check_mlp(p, obs_stride, n_units, units_per_group);
    if (rc) return rc;
    if (n_envs < 1) return fail(MS_EINVAL, "n_envs must be >= 1");
    if (n_cores < 1 || n_units % n_cores != 0) return fail(MS_EINVAL, "n_units must be n_agents * n_cores");
    if (obs_stride < 16) return fail(MS_EINVAL, "obs_stride must be >= 16");
    HIP_TRY(ms::launch_policy_act_compact(p, core_rows, core_owner, obs_stride, n_envs, n_units, units_per_group,
                                          n_cores, common_row, seed, offset, offset_dev, uniforms, action, logprob,
                                          (hipStream_t)stream));
    return MS_OK;
}

int ms_act_round_free(const ms_mlp_params* core, const ms_mlp_params* price, const int8_t* off_obs, int32_t off_stride,
                      int32_t off_units, int32_t off_units_per_group, const ms_mlp_params* acc, const int8_t* core_rows,
                      const int8_t* core_owner, int32_t acc_stride, int32_t acc_units, int32_t acc_units_per_group,
                      int32_t n_cores, const int8_t* common_row, int64_t n_envs, uint64_t seed, uint64_t off_offset,
                      uint64_t acc_offset, const uint64_t* offset_dev, int8_t* core_action, float* core_logprob,
                      int8_t* price_state, int8_t* price_action, float* price_logprob, int8_t* env_price,
                      int8_t* acc_action, float* acc_logprob, const ms_price_table* price_table,
                      int64_t price_unit_stride, void* stream) {
    if (!off_obs || !core_rows || !core_owner || !common_row || !core_action || !core_logprob || !acc_action ||
        !acc_logprob)
        return fail(MS_EINVAL, "NULL argument");
    // price == NULL: a fixed-price round (the offer units' net acts alone; no price outputs)
    if (price && (!price_state || !price_action || !price_logprob || !env_price))
        return fail(MS_EINVAL, "NULL price output");
    if (!price && (price_state || price_action || price_logprob || env_price || price_table))
        return fail(MS_EINVAL, "a fixed-price round (price_chooser NULL) takes no price outputs or table");
    if (n_envs < 1) return fail(MS_EINVAL, "n_envs must be >= 1");
    int rc = check_mlp(core, off_stride, off_units, off_units_per_group);
    if (rc) return rc;
    if (price) {
        rc = check_mlp(price, 4, off_units, off_units_per_group);
        if (rc) return rc;
    }
    rc = check_mlp(acc, acc_stride, acc_units, acc_units_per_group);
    if (rc) return rc;
    if (price && (price->in_dim != 4 || price->n_groups != core->n_groups))
        return fail(MS_EINVAL, "price chooser must be 4 -> A");
    if (core->in_dim != 2 * n_cores + 2 || core->n_actions != n_cores + 1)
        return fail(MS_EINVAL, "core chooser must be (2C+2) -> C+1");
    if (n_cores < 1 || acc_units % n_cores != 0 || acc_stride < 16)
        return fail(MS_EINVAL, "acceptor units must be n_agents * n_cores with obs_stride >= 16");
    if (price_table && (!price_table->digit || !price_table->table || price_table->n_keys < 1))
        return fail(MS_EINVAL, "price_table needs digit, table and n_keys >= 1");
    if (price_unit_stride != 0 && price_unit_stride < n_envs)
        return fail(MS_EINVAL, "price_unit_stride must be 0 or >= n_envs");
    HIP_TRY(ms::launch_act_round(core, price, off_obs, off_stride, off_units, off_units_per_group, acc, core_rows,
                                 core_owner, acc_stride, acc_units, acc_units_per_group, n_cores, common_row, n_envs,
                                 seed, off_offset, acc_offset, offset_dev, core_action, core_logprob, price_state,
                                 price_action, price_logprob, env_price, acc_action, acc_logprob,
                                 price_table ? price_table->table : nullptr, price_table ? price_table->digit : nullptr,
                                 price_table ? price_table->n_keys : 0, price_unit_stride, (hipStream_t)stream));
    return MS_OK;
}

int ms_price_table_build(const ms_mlp_params* price_chooser, const ms_price_table* t, void* stream) {
    if (!price_chooser || !t || !t->rows || !t->table || t->n_keys < 1) return fail(MS_EINVAL, "NULL argument");
    int rc = check_mlp(price_chooser, 4, price_chooser->n_groups, 1);
    if (rc) return rc;
    if (price_chooser->in_dim != 4 || price_chooser->n_actions > 32)
        return fail(MS_EINVAL, "price chooser must be 4 -> A with A <= 32");
    HIP_TRY(ms::launch_price_table(price_chooser, t->rows, t->n_keys, t->table, (hipStream_t)stream));
    return MS_OK;
}

size_t ms_act_frag_bytes(const ms_mlp_params* p, int32_t obs_stride) {
    if (!p || obs_stride < 1 || p->n_groups < 1) return 0;
    return ms::act_frag_bytes(p, obs_stride);
}

int ms_act_prepare(const ms_mlp_params* p, const int8_t* common_row, int32_t obs_stride, void* frag, void* stream) {
    if (!p || !frag) return fail(MS_EINVAL, "NULL argument");
    if (obs_stride < 4 || (obs_stride & 3)) return fail(MS_EINVAL, "obs_stride must be a positive multiple of 4");
    int rc = check_mlp(p, obs_stride, p->n_groups, 1);
    if (rc) return rc;
    HIP_TRY(ms::launch_act_prepare(p, common_row, obs_stride, frag, (hipStream_t)stream));
    return MS_OK;
}

int ms_offer_act_free(const ms_mlp_params* core, const ms_mlp_params* price, const int8_t* obs, int32_t obs_stride,
                      int64_t n_envs, int32_t n_units, int32_t units_per_group, int32_t n_cores, uint64_t seed,
                      uint64_t offset, const uint64_t* offset_dev, const float* uniforms, int8_t* core_action,
                      float* core_logprob, int8_t* price_state, int8_t* price_action, float* price_logprob,
                      int8_t* env_price, int64_t price_unit_stride, void* stream) {
    if (!obs || !core_action || !core_logprob || !price_state || !price_action || !price_logprob || !env_price)
        return fail(MS_EINVAL, "NULL argument");
    int rc = check_mlp(core, obs_stride, n_units, units_per_group);
    if (rc) return rc;
    rc = check_mlp(price, 4, n_units, units_per_group);
    if (rc) return rc;
    if (price->in_dim != 4 || price->n_groups != core->n_groups) return fail(MS_EINVAL, "price chooser must be 4 -> A");
    if (core->in_dim != 2 * n_cores + 2 || core->n_actions != n_cores + 1)
        return fail(MS_EINVAL, "core chooser must be (2C+2) -> (C+1)");
    if (n_envs < 1) return fail(MS_EINVAL, "n_envs must be >= 1");
    if (price_unit_stride != 0 && price_unit_stride < n_envs)
        return fail(MS_EINVAL, "price_unit_stride must be 0 or >= n_envs");
    HIP_TRY(ms::launch_offer_act_free(core, price, obs, obs_stride, n_envs, n_units, units_per_group, n_cores, seed,
                                      offset, offset_dev, uniforms, core_action, core_logprob, price_state,
                                      price_action, price_logprob, env_price, price_unit_stride, (hipStream_t)stream));
    return MS_OK;
}

// keyed rows (ppo_kernels.hip) for nets of at most 4 inputs and 32 actions: the byte sizes of the
// table arrays that follow the partial vectors in the workspace
static bool ppo_keyable(const ms_mlp_params* a) { return a->in_dim <= 4 && a->n_actions <= 32; }
struct KeyWs {
    size_t mark, idx, act, olp, ret, rank, sorted, n, flag, part, pcnt, ploss, fwd;
    size_t total() const {
        return align256(mark) + align256(idx) + align256(act) + align256(olp) + align256(ret) + align256(rank) +
               align256(sorted) + align256(n) + align256(flag) + align256(part) + align256(pcnt) + align256(ploss) +
               align256(fwd);
    }
    static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
};
static KeyWs key_ws(const ms_mlp_params* a, int64_t rows) {
    const size_t G = (size_t)a->n_groups, nt16 = 16 * (size_t)((a->n_actions + 15) / 16), gr = G * (size_t)rows;
    const size_t dense = G * ms::kKeyDense, ranks = G * ms::kKeyMaxRanks, pr = ranks * ms::kKeyScanBlocks;
    return KeyWs{dense, gr * 4, gr, gr * 4, gr * 4, dense * 4, ranks * 4, G * 4, G * 4, pr * (nt16 + 1) * 8, pr * 4,
                 G * ms::kKeyScanBlocks * 16, ranks * (nt16 + 4) * 4};
}
static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
static size_t ppo_partials_bytes(const ms_mlp_params* a, int64_t rows) {
    int ct, nc;
    ppo_split(rows, a->n_groups, &ct, &nc);
    return align256((size_t)a->n_groups * ms::ppo_partial_rows(nc, ppo_keyable(a)) *
                    ms::ppo_param_count(a->in_dim, a->n_actions) * sizeof(float));  // one vector per block
}

// k_own_scan's buffers (compact acceptor rows of >= kOwnMinGroups groups): the groups' row masks,
// the scan blocks' int64 sums, the scan waves' float sums, the common-row forward table and sums
struct OwnWs {
    size_t mask, part, wpart, cfwd, csum;
    int words, nb;
    size_t total() const { return KeyWs::align256(mask) + KeyWs::align256(part) + KeyWs::align256(wpart) +
                                  KeyWs::align256(cfwd) + KeyWs::align256(csum); }
};
static bool ppo_ownable(const ms_mlp_params* a) { return a->n_groups >= ms::kOwnMinGroups && a->in_dim >= 16; }
static OwnWs own_ws(const ms_mlp_params* a, int64_t rows) {
    const size_t G = (size_t)a->n_groups, A = (size_t)a->n_actions, KA = 16 * ((A + 15) / 16);
    OwnWs w{};
    w.words = (int)((rows + 31) / 32);
    w.nb = (int)((rows + 4 * ms::kOwnScanRows - 1) / (4 * ms::kOwnScanRows));
    w.mask = G * (size_t)w.words * 4;
    w.part = G * (size_t)w.nb * A * 8;
    w.wpart = G * 4 * (size_t)w.nb * 8 * 4;
    w.cfwd = G * (KA + 4) * 4;
    w.csum = G * (KA + 8) * 4;
    return w;
}

size_t ms_ppo_workspace_bytes(const ms_mlp_params* a, int64_t rows) {
    if (!a || rows < 1 || a->n_groups < 1) return 0;
    size_t b = ppo_partials_bytes(a, rows);
    if (ppo_keyable(a)) b += key_ws(a, rows).total();
    if (ppo_ownable(a)) b += own_ws(a, rows).total();
    return b;
}

int ms_ppo_grad(const ms_mlp_params* a, const ms_mlp_params* c, const ms_ppo_batch* b, float eps_clip, void* ws,
                size_t ws_bytes, const ms_ppo_grads* g, void* stream) {
    if (!a || !c || !b || !g || !ws) return fail(MS_EINVAL, "NULL argument");
    if (a->hidden != 16 || c->hidden != 16) return fail(MS_EINVAL, "hidden width must be 16");
    if (c->n_actions != 1 || c->in_dim != a->in_dim || c->n_groups != a->n_groups)
        return fail(MS_EINVAL, "critic must be [D -> 16 -> 16 -> 1] with the actor's groups");
    if (a->in_dim < 1 || a->in_dim > 256 || a->n_actions < 1 || a->n_actions > 128)
        return fail(MS_EINVAL, "in_dim must be in [1, 256] and n_actions in [1, 128]");
    if (b->stride < a->in_dim || (b->stride & 3) || b->T < 1 || b->E < 1 || b->U < 1)
        return fail(MS_EINVAL, "bad batch shape");
    if (!b->states || !b->actions || !b->old_logprobs || !b->returns || !b->unit_of_group)
        return fail(MS_EINVAL, "NULL batch pointer");
    if (b->core_owner && (!b->common_row || b->n_cores < 1 || b->U % b->n_cores != 0 || b->stride < 16))
        return fail(MS_EINVAL, "compact rows need common_row, stride >= 16 and U = n_agents * n_cores");
    const int64_t R = (int64_t)b->T * b->E;
    if (b->unit_stride != 0 && (b->unit_stride < R || b->core_owner))
        return fail(MS_EINVAL, "unit_stride must be 0 or >= T*E (and not with compact rows)");
    if (ws_bytes < ms_ppo_workspace_bytes(a, R)) return fail(MS_EINVAL, "workspace too small");
    ms::PpoArgs p{};
    p.w1 = a->w1; p.b1 = a->b1; p.w2 = a->w2; p.b2 = a->b2; p.w3 = a->w3; p.b3 = a->b3;
    p.cw1 = c->w1; p.cb1 = c->b1; p.cw2 = c->w2; p.cb2 = c->b2; p.cw3 = c->w3; p.cb3 = c->b3;
    p.states = b->states;
    p.actions = b->actions;
    p.old_lp = b->old_logprobs;
    p.rrs = b->unit_stride ? 1 : b->U;
    p.rus = b->unit_stride ? b->unit_stride : 1;
    p.ret = b->returns;
    p.unit_of_group = b->unit_of_group;
    p.common = b->common_row;
    p.owner = b->core_owner;
    p.owner_C = b->n_cores;
    p.partials = (float*)ws;
    p.D = a->in_dim;
    p.A = a->n_actions;
    p.stride = b->stride;
    p.T = b->T;
    p.U = b->U;
    p.G = a->n_groups;
    p.ret_ld = b->returns_ld > 0 ? b->returns_ld : p.G;
    p.E = b->E;
    p.R = R;
    ppo_split(R, p.G, &p.chunk_tiles, &p.n_chunks);
    p.P = ms::ppo_param_count(p.D, p.A);
    p.eps_clip = eps_clip;
    p.inv_R = 1.0f / (float)R;
    if (ppo_keyable(a) && b->row_keys == 0) {
        const KeyWs k = key_ws(a, R);
        uint8_t* w = (uint8_t*)ws + ppo_partials_bytes(a, R);
        auto take = [&w](size_t bytes) {
            uint8_t* q = w;
            w += KeyWs::align256(bytes);
            return q;
        };
        p.key_mark = take(k.mark);
        p.key_idx = (uint32_t*)take(k.idx);
        p.key_act = (int8_t*)take(k.act);
        p.key_olp = (float*)take(k.olp);
        p.key_ret = (float*)take(k.ret);
        p.key_rank = (int32_t*)take(k.rank);
        p.key_sorted = (uint32_t*)take(k.sorted);
        p.key_n = (int32_t*)take(k.n);
        p.key_flag = (int32_t*)take(k.flag);
        p.key_part = (long long*)take(k.part);
        p.key_pcnt = (uint32_t*)take(k.pcnt);
        p.key_ploss = (float*)take(k.ploss);
        p.key_fwd = (float*)take(k.fwd);
        p.key_nbs = ms::kKeyScanBlocks;
        // ranks per scan pass: the LDS sums (int64 per action + V - G, a uint32 count) in 147 KB
        p.key_cap = (147 * 1024) / ((16 * ((a->n_actions + 15) / 16) + 1) * 8 + 4);
        // |term| * kKeyFx * R < 2^62: a slot's int64 sum cannot overflow
        p.key_bound = (float)std::min(1e30, std::ldexp(1.0, 62) / ms::kKeyFx / (double)R);
    }
    if (ppo_ownable(a) && b->core_owner) {
        const OwnWs o = own_ws(a, R);
        uint8_t* w = (uint8_t*)ws + ppo_partials_bytes(a, R) + (ppo_keyable(a) ? key_ws(a, R).total() : 0);
        auto take = [&w](size_t bytes) {
            uint8_t* q = w;
            w += KeyWs::align256(bytes);
            return q;
        };
        p.own_mask = (uint32_t*)take(o.mask);
        p.own_part = (long long*)take(o.part);
        p.own_wpart = (float*)take(o.wpart);
        p.own_cfwd = (float*)take(o.cfwd);
        p.own_csum = (float*)take(o.csum);
        p.own_words = o.words;
        p.own_nb = o.nb;
        // |term| * 2^28 * R < 2^63: the group's int64 sum over all its rows cannot overflow
        p.own_qbound = (float)std::min(1e30, std::ldexp(1.0, 35) / (double)R);
    }
    ms::GradOut go{g->w1, g->b1, g->w2, g->b2, g->w3, g->b3, g->cw1, g->cb1, g->cw2, g->cb2, g->cw3, g->cb3, g->loss};
    HIP_TRY(ms::launch_ppo_grad(p, go, (hipStream_t)stream));
    return MS_OK;
}

int ms_aggregate_obs(const ms_config* cfg, int64_t E, const int8_t* acc_obs, const int8_t* off_obs,
                     int8_t* agg_acceptor, int8_t* agg_offer, int8_t* fully, void* stream) {
    int rc = validate_config(cfg);
    if (rc) return rc;
    if (E < 1 || !acc_obs || !off_obs) return fail(MS_EINVAL, "need E >= 1 and both divided observation arrays");
    const ms::Params P = ms::make_params(*cfg, cap_of(cfg));
    ms::AggArgs g{};
    g.acc = acc_obs;
    g.off = off_obs;
    g.out_acc = agg_acceptor;
    g.out_off = agg_offer;
    g.out_full = fully;
    g.N = P.N;
    g.C = P.C;
    g.L = P.L;
    g.d_acc = P.d_acc;
    g.acc_stride = P.acc_stride;
    g.off_stride = P.off_stride;
    g.agg_acc_stride = ms::align4(P.C * P.d_acc);
    g.agg_off_stride = ms::align4(2 * P.C + 2 * P.L);
    g.full_stride = ms::align4(2 * P.C + 2 * P.L + P.C * P.d_acc);
    g.E = E;
    HIP_TRY(ms::launch_aggregate_obs(g, (hipStream_t)stream));
    return MS_OK;
}

int ms_decode_aggregated(const ms_config* cfg, int64_t E, const int32_t* actions, int32_t fully, int8_t* acceptor,
                         int8_t* offer_core, int32_t* n_bad, void* stream) {
    int rc = validate_config(cfg);
    if (rc) return rc;
    if (E < 1 || !actions || !acceptor || !offer_core) return fail(MS_EINVAL, "NULL argument or E < 1");
    const ms::Params P = ms::make_params(*cfg, cap_of(cfg));
    double space = 1.0;
    for (int c = 0; c < P.C; c++) space *= (double)(P.O + 1);
    for (int s = 0; s < P.L; s++) space *= (double)(P.C + 1);
    if (space > 2147483647.0) return fail(MS_EINVAL, "aggregated action space (O+1)^C * (C+1)^L exceeds int32");
    HIP_TRY(ms::launch_decode_aggregated(actions, (long long)E * P.N, P.C, P.L, P.O, fully ? 1 : 0, acceptor,
                                         offer_core, n_bad, (hipStream_t)stream));
    return MS_OK;
}

static_assert(sizeof(ms_adam_tensor) == sizeof(ms::AdamTensor), "ms_adam_tensor layout");
static_assert(MS_ADAM_MAX_TENSORS == ms::kAdamMaxTensors, "ms_adam_tensor count");

int ms_adam_step(const ms_adam_tensor* tensors, int32_t n_tensors, const double* lr, int32_t n_lr, int64_t step,
                 double beta1, double beta2, double eps, void* stream) {
    if (!tensors || !lr) return fail(MS_EINVAL, "NULL argument");
    if (n_tensors < 1 || n_tensors > MS_ADAM_MAX_TENSORS) return fail(MS_EINVAL, "n_tensors must be in [1, %d]", MS_ADAM_MAX_TENSORS);
    if (n_lr < 1 || n_lr > ms::kAdamMaxGroups) return fail(MS_EINVAL, "n_lr must be in [1, %d]", ms::kAdamMaxGroups);
    if (step < 1) return fail(MS_EINVAL, "step must be >= 1");
    for (int i = 0; i < n_tensors; i++) {
        const ms_adam_tensor& t = tensors[i];
        if (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq || t.numel < 0) return fail(MS_EINVAL, "bad tensor %d", i);
        if (t.lr_group < 0 || t.lr_group >= n_lr) return fail(MS_EINVAL, "tensor %d: lr_group out of range", i);
    }
    HIP_TRY(ms::launch_adam(reinterpret_cast<const ms::AdamTensor*>(tensors), n_tensors, lr, n_lr, step, beta1, beta2,
                            eps, nullptr, (hipStream_t)stream));
    return MS_OK;
}

int ms_adam_step_dev(const ms_adam_tensor* tensors, int32_t n_tensors, const double* lr, int32_t n_lr,
                     const int64_t* step_dev, double beta1, double beta2, double eps, void* stream) {
    if (!tensors || !lr || !step_dev) return fail(MS_EINVAL, "NULL argument");
    if (n_tensors < 1 || n_tensors > MS_ADAM_MAX_TENSORS) return fail(MS_EINVAL, "n_tensors must be in [1, %d]", MS_ADAM_MAX_TENSORS);
    if (n_lr < 1 || n_lr > ms::kAdamMaxGroups) return fail(MS_EINVAL, "n_lr must be in [1, %d]", ms::kAdamMaxGroups);
    for (int i = 0; i < n_tensors; i++) {
        const ms_adam_tensor& t = tensors[i];
        if (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq || t.numel < 0) return fail(MS_EINVAL, "bad tensor %d", i);
        if (t.lr_group < 0 || t.lr_group >= n_lr) return fail(MS_EINVAL, "tensor %d: lr_group out of range", i);
    }
    HIP_TRY(ms::launch_adam(reinterpret_cast<const ms::AdamTensor*>(tensors), n_tensors, lr, n_lr, 0, beta1, beta2, eps,
                            step_dev, (hipStream_t)stream));
    return MS_OK;
}

int ms_unit_returns(const void* rewards, int32_t rewards_i32, int32_t T, int64_t E, int32_t U,
                    const int32_t* unit_of_group, int32_t G, double gamma, float* out, void* stream) {
    if (!rewards || !unit_of_group || !out) return fail(MS_EINVAL, "NULL argument");
    if (T < 1 || E < 0 || U < 1 || G < 1) return fail(MS_EINVAL, "bad shape");
    HIP_TRY(ms::launch_unit_returns(rewards, rewards_i32 ? 1 : 0, T, E, U, unit_of_group, G, gamma, out,
                                    (hipStream_t)stream));
    return MS_OK;
}

int ms_discounted_returns(const float* rewards, int32_t T, int64_t M, int64_t row_stride, double gamma, float* out,
                          void* stream) {
    if (!rewards || !out) return fail(MS_EINVAL, "NULL argument");
    if (T < 1 || M < 0 || row_stride < M) return fail(MS_EINVAL, "bad shape");
    HIP_TRY(ms::launch_returns(rewards, T, M, row_stride, gamma, out, (hipStream_t)stream));
    return MS_OK;
}

}  // extern "C"

// ---- DQN units

static int qnet_check(const ms_qnet_params* q, const char* who) {
    if (!q || !q->w1 || !q->b1 || !q->w2 || !q->b2) return fail(MS_EINVAL, "%s: null net parameter", who);
    if (q->hidden != ms::kQH) return fail(MS_EINVAL, "%s: hidden must be %d", who, ms::kQH);
    if (q->in_dim < 1 || q->in_dim > 256 || q->n_actions < 1 || q->n_actions > 127 || q->n_groups < 1)
        return fail(MS_EINVAL, "%s: bad net shape", who);
    return MS_OK;
}

static ms::QArgs qargs(const ms_qnet_params* q, int upg) {
    ms::QArgs a;
    a.w1 = q->w1;
    a.b1 = q->b1;
    a.w2 = q->w2;
    a.b2 = q->b2;
    a.D = q->in_dim;
    a.A = q->n_actions;
    a.G = q->n_groups;
    a.upg = upg;
    return a;
}

static int dqn_param_count(int D, int A) { return ms::kQH * D + ms::kQH + A * ms::kQH + A; }

int ms_dqn_act(const ms_qnet_params* q, const int8_t* obs, int32_t obs_stride, int64_t n_envs, int32_t n_units,
               int32_t units_per_group, double eps_threshold, const double* uniforms, uint64_t seed, uint64_t offset,
               const uint64_t* offset_dev, int8_t* action, int8_t* greedy, void* stream) {
    if (int rc = qnet_check(q, "ms_dqn_act")) return rc;
    if (!obs || !action || n_envs < 1 || n_units < 1 || units_per_group < 1 ||
        units_per_group * q->n_groups != n_units || obs_stride < q->in_dim || (obs_stride & 3))
        return fail(MS_EINVAL, "ms_dqn_act: bad rows / units (units_per_group * n_groups must equal n_units)");
    if (n_units > 65535) return fail(MS_EINVAL, "ms_dqn_act: at most 65535 units");
    ms::DqnActArgs a{};
    a.q = qargs(q, units_per_group);
    a.obs = obs;
    a.stride = obs_stride;
    a.U = n_units;
    a.E = n_envs;
    a.eps = eps_threshold;
    a.uniforms = uniforms;
    a.seed = seed;
    a.offset = offset;
    a.offset_dev = offset_dev;
    a.action = action;
    a.greedy = greedy;
    HIP_TRY(ms::launch_dqn_act(a, (hipStream_t)stream));
    return MS_OK;
}

static int dqn_xpitch(int D) { return 4 * ((((D + 3) / 4)) | 1); }

size_t ms_dqn_workspace_bytes(const ms_qnet_params* q, int64_t rows_per_group) {
    if (!q || rows_per_group < 1) return 0;
    const int64_t nblk = (rows_per_group + 255) / 256;
    return sizeof(float) * (size_t)q->n_groups * (size_t)nblk * (size_t)(dqn_param_count(q->in_dim, q->n_actions) + 1);
}

int ms_dqn_grad(const ms_qnet_params* policy, const ms_qnet_params* target, const ms_dqn_batch* b, float grad_clip,
                void* workspace, size_t workspace_bytes, const ms_qnet_grads* g, void* stream) {
    if (int rc = qnet_check(policy, "ms_dqn_grad (policy)")) return rc;
    if (int rc = qnet_check(target, "ms_dqn_grad (target)")) return rc;
    if (policy->in_dim != target->in_dim || policy->n_actions != target->n_actions ||
        policy->n_groups != target->n_groups)
        return fail(MS_EINVAL, "ms_dqn_grad: policy and target shapes differ");
    if (!b || !g || !b->states || !b->next_states || !b->actions || !b->rewards || !b->samples || !g->w1 || !g->b1 ||
        !g->w2 || !g->b2 || !g->loss)
        return fail(MS_EINVAL, "ms_dqn_grad: null batch / gradient pointer");
    if (b->n_envs < 1 || b->batch < 1 || b->capacity < 1 || b->units_per_group < 1 ||
        b->units_per_group * policy->n_groups != b->n_units || b->stride < policy->in_dim || (b->stride & 3))
        return fail(MS_EINVAL, "ms_dqn_grad: bad batch shape");
    const int64_t rows = (int64_t)b->units_per_group * b->n_envs * b->batch;
    const size_t need = ms_dqn_workspace_bytes(policy, rows);
    if (!workspace || workspace_bytes < need) return fail(MS_EINVAL, "ms_dqn_grad: workspace too small (%zu < %zu)",
                                                          workspace_bytes, need);
    ms::DqnGradArgs a{};
    a.q = qargs(policy, b->units_per_group);
    a.t = qargs(target, b->units_per_group);
    a.states = b->states;
    a.next_states = b->next_states;
    a.actions = b->actions;
    a.rewards = b->rewards;
    a.samples = b->samples;
    a.stride = b->stride;
    a.U = b->n_units;
    a.cap = b->capacity;
    a.B = b->batch;
    a.xpitch = dqn_xpitch(policy->in_dim);
    a.P = dqn_param_count(policy->in_dim, policy->n_actions) + 1;
    a.E = b->n_envs;
    a.rows = rows;
    a.gamma = b->gamma;
    a.inv_rows = (float)(1.0 / (double)rows);
    a.partials = static_cast<float*>(workspace);
    if (ms::dqn_grad_lds(a.q, a.xpitch) > 160 * 1024) return fail(MS_EINVAL, "ms_dqn_grad: net too wide for LDS");
    ms::DqnReduceArgs r{};
    r.partials = a.partials;
    r.nblk = (int)((rows + 255) / 256);
    r.P = a.P;
    r.D = a.q.D;
    r.A = a.q.A;
    r.clip = grad_clip;
    r.inv_rows = a.inv_rows;
    r.w1 = g->w1;
    r.b1 = g->b1;
    r.w2 = g->w2;
    r.b2 = g->b2;
    r.loss = g->loss;
    if (r.nblk > 65535 * 64) return fail(MS_EINVAL, "ms_dqn_grad: too many rows per group");
    HIP_TRY(ms::launch_dqn_grad(a, r, (hipStream_t)stream));
    return MS_OK;
}

int ms_regen_agent_rows(const ms_config* cfg, const int8_t* core_rows, const int8_t* core_owner,
                        const int8_t* slot_pairs, const int64_t* frame, const int32_t* agent, int64_t n_rows,
                        int8_t* acceptor, int8_t* offer, void* stream) {
    int rc = validate_config(cfg);
    if (rc) return rc;
    if (n_rows < 0 || !frame || !agent || !core_rows) return fail(MS_EINVAL, "ms_regen_agent_rows: NULL argument");
    if (!acceptor && !offer) return MS_OK;
    if (acceptor && !core_owner) return fail(MS_EINVAL, "ms_regen_agent_rows: acceptor rows need core_owner");
    if (offer && !slot_pairs) return fail(MS_EINVAL, "ms_regen_agent_rows: offer rows need slot_pairs");
    const ms::Params P = ms::make_params(*cfg, cap_of(cfg));
    ms::RegenArgs g{};
    g.core_rows = core_rows;
    g.core_owner = core_owner;
    g.slot_pairs = slot_pairs;
    g.frame = frame;
    g.agent = agent;
    g.acc = acceptor;
    g.off = offer;
    g.n = n_rows;
    g.N = P.N;
    g.C = P.C;
    g.L = P.L;
    g.d_acc = P.d_acc;
    g.acc_stride = P.acc_stride;
    g.acc_ld = ms::align4(P.C * P.d_acc);
    g.off_ld = ms::align4(2 * P.C + 2 * P.L);
    HIP_TRY(ms::launch_regen_agent_rows(g, (hipStream_t)stream));
    return MS_OK;
}

// ---- Branching DQN acting (bdqn_kernels.hip)
static int bdqn_pad(int seg) { return (seg + 31) & ~31; }

// prepared layer 1: the split W1 [3][128][segs][Dp] bf16, then cF [segs][128] f32 (W1_c F, compact acting)
static size_t bdqn_split_bytes(int32_t seg, int32_t segs) {
    return (size_t)3 * ms::kBH * segs * bdqn_pad(seg) * sizeof(uint16_t);
}
size_t ms_bdqn_workspace_bytes(int32_t seg, int32_t segs) {
    if (seg < 1 || segs < 1) return 0;
    return bdqn_split_bytes(seg, segs) + (size_t)segs * ms::kBH * sizeof(float);
}

static int bdqn_check(const ms_bdqn_params* q, const char* who) {
    if (!q || !q->w1 || !q->b1 || !q->w2 || !q->b2 || !q->wv || !q->bv || !q->wa || !q->ba)
        return fail(MS_EINVAL, "%s: NULL parameter", who);
    if (q->obs < 1 || q->ac_dim < 1 || q->ac_dim > 127 || q->n < 1 || q->n > 128)
        return fail(MS_EINVAL, "%s: bad net shape (obs %d, ac_dim %d, n %d)", who, q->obs, q->ac_dim, q->n);
    return MS_OK;
}

static ms::BdqnNet bdqn_net(const ms_bdqn_params* q) {
    return ms::BdqnNet{q->w1, q->b1, q->w2, q->b2, q->wv, q->bv, q->wa, q->ba, q->obs, q->ac_dim, q->n};
}

// update_policy workspace (bdqn_update_kernels.hip): layer-1 partials [3][nK][128][128]; the rows'
// activations and pre-activation gradients [6][128][128] (out1, out2 x 3, dpre2, dpre1); head outputs
// [3][128][Mp]; head gradients [128][Mp]; d out2 partials [Mp/64][128][128]; the rows' losses
struct BdqnUpdWs {
    int nK, Mp;
    size_t l1p, rows, q3, dq, d2p, small, total;
};
static BdqnUpdWs bdqn_upd_ws(const ms_bdqn_params* q) {
    BdqnUpdWs w{};
    w.nK = (q->obs + 127) / 128;
    w.Mp = (q->ac_dim * q->n + 1 + 63) / 64 * 64;
    w.l1p = align256(sizeof(float) * 3 * (size_t)w.nK * 128 * 128);
    w.rows = align256(sizeof(float) * 6 * 128 * 128);
    w.q3 = align256(sizeof(float) * 3 * 128 * (size_t)w.Mp);
    w.dq = align256(sizeof(float) * 128 * (size_t)w.Mp);
    w.d2p = align256(sizeof(float) * (size_t)(w.Mp / 64) * 128 * 128);
    w.small = align256(sizeof(float) * 128);
    w.total = w.l1p + w.rows + w.q3 + w.dq + w.d2p + w.small;
    return w;
}

size_t ms_bdqn_update_workspace_bytes(const ms_bdqn_params* q, int32_t batch) {
    if (!q || batch < 1 || batch > 128 || q->obs < 1 || q->ac_dim < 1 || q->n < 1) return 0;
    return bdqn_upd_ws(q).total;
}

int ms_bdqn_update(const ms_bdqn_params* q, const ms_bdqn_params* target, const ms_bdqn_batch* b, float gamma,
                   float grad_clip, void* ws, size_t ws_bytes, const ms_bdqn_grads* g, void* stream) {
    if (int rc = bdqn_check(q, "ms_bdqn_update")) return rc;
    if (int rc = bdqn_check(target, "ms_bdqn_update (target)")) return rc;
    if (!b || !g || !ws) return fail(MS_EINVAL, "ms_bdqn_update: NULL argument");
    if (target->obs != q->obs || target->ac_dim != q->ac_dim || target->n != q->n)
        return fail(MS_EINVAL, "ms_bdqn_update: target shape differs from the online net");
    if (q->ac_dim > 32) return fail(MS_EINVAL, "ms_bdqn_update: ac_dim %d > 32", q->ac_dim);
    if (b->batch < 1 || b->batch > 128 || !b->states || !b->next_states || !b->actions || !b->rewards || !b->masks ||
        b->ld < q->obs || b->actions_ld < q->ac_dim)
        return fail(MS_EINVAL, "ms_bdqn_update: bad batch (1..128 rows, ld >= obs, actions_ld >= ac_dim)");
    if (!g->w1 || !g->b1 || !g->w2 || !g->b2 || !g->wv || !g->bv || !g->wa || !g->ba || !g->loss)
        return fail(MS_EINVAL, "ms_bdqn_update: NULL gradient tensor");
    const BdqnUpdWs w = bdqn_upd_ws(q);
    if (w.Mp > ms::kUpdMaxHeadRows)
        return fail(MS_EINVAL, "ms_bdqn_update: ac_dim * n + 1 = %d head rows > %d", q->ac_dim * q->n + 1,
                    ms::kUpdMaxHeadRows);
    if (ws_bytes < w.total) return fail(MS_EINVAL, "ms_bdqn_update: workspace too small (%zu < %zu)", ws_bytes, w.total);
    ms::BdqnUpd p{};
    p.q = bdqn_net(q);
    p.t = bdqn_net(target);
    p.xs = b->states;
    p.xn = b->next_states;
    p.ld = b->ld;
    p.act = b->actions;
    p.act_ld = b->actions_ld;
    p.rew = b->rewards;
    p.mask = b->masks;
    p.B = b->batch;
    p.gamma = gamma;
    p.clip = grad_clip > 0.f ? grad_clip : 3.0e38f;
    p.nK = w.nK;
    p.Mp = w.Mp;
    char* base = (char*)ws;
    p.l1p = (float*)base;
    float* rows = (float*)(base + w.l1p);
    p.out1 = rows;
    p.out2 = rows + 128 * 128;
    p.dpre2 = rows + 4 * 128 * 128;
    p.dpre1 = rows + 5 * 128 * 128;
    size_t off = w.l1p + w.rows;
    p.q3 = (float*)(base + off);
    off += w.q3;
    p.dq = (float*)(base + off);
    off += w.dq;
    p.d2p = (float*)(base + off);
    off += w.d2p;
    p.lossb = (float*)(base + off);
    p.g = ms::BdqnGrads{g->w1, g->b1, g->w2, g->b2, g->wv, g->bv, g->wa, g->ba, g->loss};
    HIP_TRY(ms::launch_bdqn_update(p, (hipStream_t)stream));
    return MS_OK;
}

int ms_bdqn_prepare(const ms_bdqn_params* q, int32_t seg, int32_t segs, void* workspace, size_t workspace_bytes,
                    float* base, void* stream) {
    if (int rc = bdqn_check(q, "ms_bdqn_prepare")) return rc;
    if (seg < 1 || segs < 1 || (int64_t)seg * segs != q->obs)
        return fail(MS_EINVAL, "ms_bdqn_prepare: seg * segs must equal obs");
    if (!workspace || workspace_bytes < ms_bdqn_workspace_bytes(seg, segs))
        return fail(MS_EINVAL, "ms_bdqn_prepare: workspace too small");
    HIP_TRY(ms::launch_bdqn_w1split(q->w1, seg, segs, bdqn_pad(seg), (uint16_t*)workspace, (hipStream_t)stream));
    if (base)
        HIP_TRY(ms::launch_bdqn_l1_base(q->w1, q->b1, seg, segs, (float*)((char*)workspace + bdqn_split_bytes(seg, segs)),
                                        base, (hipStream_t)stream));
    return MS_OK;
}

// compact layer-1 scratch: P [E][C][128] f32, then (ms_bdqn_act_compact) the owning-row count, the
// common row's actions and the row list [1 + E * 127] int32
static size_t bdqn_p_bytes(int64_t n_envs, int32_t n_cores) {
    return align256(sizeof(float) * (size_t)n_envs * n_cores * ms::kBH);
}
size_t ms_bdqn_layer1_scratch_bytes(int64_t n_envs, int32_t n_cores) {
    if (n_envs < 1 || n_cores < 1) return 0;
    return bdqn_p_bytes(n_envs, n_cores) + 256 + 256 + align256(sizeof(uint64_t) * (size_t)n_envs) +
           sizeof(int32_t) * (1 + (size_t)n_envs * 127);
}

int ms_bdqn_layer1_compact(const ms_bdqn_params* q, const void* workspace, const float* base, const int8_t* core_rows,
                           const int8_t* core_owner, int64_t n_envs, int32_t n_agents, int32_t n_cores,
                           int32_t acc_dim, int32_t acc_stride, void* scratch, size_t scratch_bytes, float* h1,
                           void* stream) {
    if (int rc = bdqn_check(q, "ms_bdqn_layer1_compact")) return rc;
    if (!workspace || !base || !core_rows || !core_owner || !h1 || !scratch)
        return fail(MS_EINVAL, "ms_bdqn_layer1_compact: NULL argument");
    if (n_envs < 1 || n_agents < 1 || n_agents > 127 || n_cores < 1 || acc_dim < 4 || acc_dim > 256 ||
        acc_stride < acc_dim || (acc_stride & 3) || (int64_t)acc_dim * n_cores != q->obs)
        return fail(MS_EINVAL, "ms_bdqn_layer1_compact: bad shape (obs must be n_cores * acc_dim)");
    if (scratch_bytes < ms_bdqn_layer1_scratch_bytes(n_envs, n_cores))
        return fail(MS_EINVAL, "ms_bdqn_layer1_compact: scratch too small");
    ms::BdqnL1Compact p{};
    p.w1s = (const uint16_t*)workspace;
    p.base = base;
    p.cF = (const float*)((const char*)workspace + bdqn_split_bytes(acc_dim, n_cores));
    p.core_rows = core_rows;
    p.core_owner = core_owner;
    p.E = n_envs;
    p.N = n_agents;
    p.C = n_cores;
    p.D = acc_dim;
    p.Dp = bdqn_pad(acc_dim);
    p.stride = acc_stride;
    p.P = (float*)scratch;
    p.h1 = h1;
    HIP_TRY(ms::launch_bdqn_l1_compact(p, (hipStream_t)stream));
    return MS_OK;
}

int ms_bdqn_act_compact(const ms_bdqn_params* q, const void* workspace, const float* base, const int8_t* core_rows,
                        const int8_t* core_owner, int64_t n_envs, int32_t n_agents, int32_t n_cores, int32_t acc_dim,
                        int32_t acc_stride, void* scratch, size_t scratch_bytes, const uint8_t* explore,
                        const int8_t* rand_action, int8_t* action, void* stream) {
    if (int rc = bdqn_check(q, "ms_bdqn_act_compact")) return rc;
    if (!workspace || !base || !core_rows || !core_owner || !scratch || !action)
        return fail(MS_EINVAL, "ms_bdqn_act_compact: NULL argument");
    if (explore && !rand_action) return fail(MS_EINVAL, "ms_bdqn_act_compact: explore needs rand_action");
    if (n_agents > 64) return fail(MS_EINVAL, "ms_bdqn_act_compact: %d agents > 64", n_agents);
    if (n_envs < 1 || n_agents < 1 || n_agents > 127 || n_cores < 1 || acc_dim < 4 || acc_dim > 256 ||
        acc_stride < acc_dim || (acc_stride & 3) || (int64_t)acc_dim * n_cores != q->obs)
        return fail(MS_EINVAL, "ms_bdqn_act_compact: bad shape (obs must be n_cores * acc_dim)");
    if (scratch_bytes < ms_bdqn_layer1_scratch_bytes(n_envs, n_cores))
        return fail(MS_EINVAL, "ms_bdqn_act_compact: scratch too small");
    ms::BdqnL1Compact l{};
    l.w1s = (const uint16_t*)workspace;
    l.base = base;
    l.cF = (const float*)((const char*)workspace + bdqn_split_bytes(acc_dim, n_cores));
    l.core_rows = core_rows;
    l.core_owner = core_owner;
    l.E = n_envs;
    l.N = n_agents;
    l.C = n_cores;
    l.D = acc_dim;
    l.Dp = bdqn_pad(acc_dim);
    l.stride = acc_stride;
    l.P = (float*)scratch;
    l.h1 = nullptr;  // the act kernel sums the P rows
    HIP_TRY(ms::launch_bdqn_l1_compact(l, (hipStream_t)stream));
    ms::BdqnAct p{};
    p.q = bdqn_net(q);
    p.rows = n_envs * n_agents;
    p.explore = explore;
    p.rnd = rand_action;
    p.action = action;
    p.P = l.P;
    p.base = base;
    p.core_owner = core_owner;
    p.N = n_agents;
    p.C = n_cores;
    // only the rows of agents owning a core run the kernel; the others take the common row's actions
    char* tail = (char*)scratch + bdqn_p_bytes(n_envs, n_cores);
    p.n_owning = (const int32_t*)tail;
    p.common = (int8_t*)(tail + 256);
    p.own_mask = (unsigned long long*)(tail + 512);
    p.list = (const int32_t*)(tail + 512 + align256(sizeof(uint64_t) * (size_t)n_envs));
    HIP_TRY(ms::launch_bdqn_act(p, (hipStream_t)stream));
    return MS_OK;
}

int ms_bdqn_act(const ms_bdqn_params* q, const float* h1, const int8_t* x, int32_t x_stride, const void* workspace,
                int64_t n_rows, const uint8_t* explore, const int8_t* rand_action, int8_t* action, void* stream) {
    if (int rc = bdqn_check(q, "ms_bdqn_act")) return rc;
    if (n_rows < 1 || !action) return fail(MS_EINVAL, "ms_bdqn_act: no rows / no action buffer");
    if (explore && !rand_action) return fail(MS_EINVAL, "ms_bdqn_act: explore needs rand_action");
    if (!h1 && (!x || !workspace || x_stride < q->obs || (x_stride & 3) || q->obs > 256))
        return fail(MS_EINVAL, "ms_bdqn_act: without h1, int8 rows (x_stride >= obs, multiple of 4, obs <= 256) "
                               "and the prepared workspace are needed");
    ms::BdqnAct p{};
    p.q = bdqn_net(q);
    p.h1 = h1;
    p.x = x;
    p.w1s = (const uint16_t*)workspace;
    p.x_stride = x_stride;
    p.Kp = bdqn_pad(q->obs);
    p.rows = n_rows;
    p.explore = explore;
    p.rnd = rand_action;
    p.action = action;
    HIP_TRY(ms::launch_bdqn_act(p, (hipStream_t)stream));
    return MS_OK;
}

// ---- wide nets: the aggregated agents' ActorCritics (wide_kernels.hip)
static int wide_check(const ms_mlp_params* a, const char* who) {
    if (!a || !a->w1 || !a->b1 || !a->w2 || !a->b2 || !a->w3 || !a->b3) return fail(MS_EINVAL, "%s: NULL parameter", who);
    if (a->hidden != 32 && a->hidden != 64) return fail(MS_EINVAL, "%s: hidden width %d not built (32, 64)", who, a->hidden);
    if (a->in_dim < 1 || a->in_dim > 255 || a->n_actions < 1 || a->n_actions > (1 << 24) || a->n_groups < 1)
        return fail(MS_EINVAL, "%s: in_dim must be in [1, 255], n_actions in [1, 2^24], n_groups >= 1", who);
    return MS_OK;
}

static ms::WideNet wide_net(const ms_mlp_params* a) { return ms::WideNet{a->w1, a->b1, a->w2, a->b2, a->w3, a->b3}; }

int ms_wide_act(const ms_mlp_params* a, const int8_t* obs, int32_t obs_stride, int64_t n_rows, const float* uniforms,
                int32_t* action, float* logprob, void* stream) {
    if (int rc = wide_check(a, "ms_wide_act")) return rc;
    if (!obs || !uniforms || !action || !logprob) return fail(MS_EINVAL, "ms_wide_act: NULL argument");
    if (n_rows < 1 || obs_stride < a->in_dim || (obs_stride & 3))
        return fail(MS_EINVAL, "ms_wide_act: n_rows >= 1 and obs_stride >= in_dim, multiple of 4");
    if ((n_rows + 15) / 16 > 0x7fffffffLL || a->n_groups > 65535) return fail(MS_EINVAL, "ms_wide_act: grid too large");
    ms::WideAct p{};
    p.actor = wide_net(a);
    p.D = a->in_dim;
    p.H = a->hidden;
    p.A = a->n_actions;
    p.G = a->n_groups;
    p.obs = obs;
    p.stride = obs_stride;
    p.E = n_rows;
    p.uniforms = uniforms;
    p.action = action;
    p.logprob = logprob;
    HIP_TRY(ms::launch_wide_act(p, (hipStream_t)stream));
    return MS_OK;
}

// work split and workspace layout of ms_wide_grad: NB row-tile blocks per group (k_wide_rows), RS
// row splits of the weight-gradient reductions (partials [RS][G][total], at most 1 GiB)
struct WidePlan {
    int NB, RS;
    long long rps;
    ms::WideOffsets off;
    size_t zbuf, rec, part, loss;  // byte offsets
    size_t bytes;
};
static WidePlan wide_plan(const ms_mlp_params* a, int64_t rows) {
    const long long R = rows;
    WidePlan w{};
    const long long H = a->hidden, D = a->in_dim, A = a->n_actions, G = a->n_groups;
    const long long cnt[ms::kWideSegs] = {H * D, H, H * H, H, A * H, A, H * D, H, H * H, H, H, 1};
    w.off.o[0] = 0;
    for (int i = 0; i < ms::kWideSegs; i++) w.off.o[i + 1] = w.off.o[i] + cnt[i];
    const long long total = w.off.o[ms::kWideSegs];
    const long long tiles = (R + 15) / 16;
    const long long nb_cap = std::max(1LL, 2048 / G);
    w.NB = (int)std::min(tiles, nb_cap);
    long long rs = std::min(64LL, std::max(1LL, (R + 255) / 256));
    const long long rs_mem = std::max(1LL, (1LL << 28) / (G * total));
    rs = std::min(rs, rs_mem);
    w.rps = ((R + rs - 1) / rs + 15) / 16 * 16;
    w.RS = (int)((R + w.rps - 1) / w.rps);
    const long long RW = 8 * H + ms::kWideStats;
    size_t o = 0;
    w.zbuf = o;
    o += align256(sizeof(float) * (size_t)(G * w.NB * 16 * A));
    w.rec = o;
    o += align256(sizeof(float) * (size_t)(G * R * RW));
    w.part = o;
    o += align256(sizeof(float) * (size_t)(w.RS * G * total));
    w.loss = o;
    o += align256(sizeof(float) * (size_t)(G * w.NB * 3));
    w.bytes = o;
    return w;
}

// The gradient workspace grows with the action count (per-block logit tiles zbuf [G][NB][16][A]);
// nets whose workspace would pass this bound are refused instead of asking for terabytes.
constexpr size_t kWideWorkspaceCap = size_t(64) << 30;

size_t ms_wide_workspace_bytes(const ms_mlp_params* a, int64_t rows) {
    if (!a || rows < 1 || a->n_groups < 1 || a->n_actions < 1 || a->in_dim < 1 ||
        (a->hidden != 32 && a->hidden != 64))
        return 0;
    const size_t b = wide_plan(a, rows).bytes;
    if (b > kWideWorkspaceCap) {
        fail(MS_EINVAL, "ms_wide_workspace_bytes: %zu bytes for %d actions exceeds the 64 GiB bound", b, a->n_actions);
        return 0;
    }
    return b;
}

int ms_wide_grad(const ms_mlp_params* a, const ms_mlp_params* c, const ms_wide_batch* b, float eps_clip, void* ws,
                 size_t ws_bytes, const ms_ppo_grads* g, void* stream) {
    if (int rc = wide_check(a, "ms_wide_grad")) return rc;
    if (!c || !b || !g || !ws) return fail(MS_EINVAL, "ms_wide_grad: NULL argument");
    if (!c->w1 || !c->b1 || !c->w2 || !c->b2 || !c->w3 || !c->b3 || c->hidden != a->hidden || c->n_actions != 1 ||
        c->in_dim != a->in_dim || c->n_groups != a->n_groups)
        return fail(MS_EINVAL, "ms_wide_grad: critic must be [D -> H -> H -> 1] with the actor's groups");
    if (!b->states || !b->actions || !b->old_logprob || !b->returns || b->rows < 1 || b->stride < a->in_dim ||
        (b->stride & 3))
        return fail(MS_EINVAL, "ms_wide_grad: bad batch (rows >= 1, stride >= in_dim, multiple of 4)");
    if (a->n_groups > 65535) return fail(MS_EINVAL, "ms_wide_grad: too many groups");
    float* dst[ms::kWideSegs] = {g->w1, g->b1, g->w2, g->b2, g->w3, g->b3, g->cw1, g->cb1, g->cw2, g->cb2, g->cw3, g->cb3};
    for (float* d : dst)
        if (!d) return fail(MS_EINVAL, "ms_wide_grad: NULL gradient tensor");
    if (!g->loss) return fail(MS_EINVAL, "ms_wide_grad: NULL loss buffer");
    const WidePlan w = wide_plan(a, b->rows);
    if (w.bytes > kWideWorkspaceCap)
        return fail(MS_EINVAL, "ms_wide_grad: workspace of %zu bytes for %d actions exceeds the 64 GiB bound", w.bytes,
                    a->n_actions);
    if (ws_bytes < w.bytes) return fail(MS_EINVAL, "ms_wide_grad: workspace too small (%zu < %zu)", ws_bytes, w.bytes);
    char* base = (char*)ws;
    ms::WideRows r{};
    r.actor = wide_net(a);
    r.critic = wide_net(c);
    r.D = a->in_dim;
    r.H = a->hidden;
    r.A = a->n_actions;
    r.G = a->n_groups;
    r.states = b->states;
    r.stride = b->stride;
    r.R = b->rows;
    r.actions = b->actions;
    r.old_logprob = b->old_logprob;
    r.returns = b->returns;
    r.eps_clip = eps_clip;
    r.inv_R = (float)(1.0 / (double)b->rows);
    r.NB = w.NB;
    r.zbuf = (float*)(base + w.zbuf);
    r.rec = (float*)(base + w.rec);
    r.loss_part = (float*)(base + w.loss);
    ms::WideGrads gp{};
    gp.actor = r.actor;
    gp.critic = r.critic;
    gp.D = r.D;
    gp.H = r.H;
    gp.A = r.A;
    gp.G = r.G;
    gp.states = b->states;
    gp.stride = b->stride;
    gp.R = b->rows;
    gp.RS = w.RS;
    gp.rows_per_split = w.rps;
    gp.rec = r.rec;
    gp.part = (float*)(base + w.part);
    gp.off = w.off;
    ms::WideReduce rp{};
    rp.part = gp.part;
    rp.RS = w.RS;
    rp.G = r.G;
    rp.NB = w.NB;
    rp.off = w.off;
    for (int i = 0; i < ms::kWideSegs; i++) rp.dst[i] = dst[i];
    rp.loss_part = r.loss_part;
    rp.loss = g->loss;
    rp.inv_R = r.inv_R;
    HIP_TRY(ms::launch_wide_grad(r, gp, rp, (hipStream_t)stream));
    return MS_OK;
}
