/*
 * ms_oracle.h — CPU restatement of the marl-scheduling environment step.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (libmarlsched.so, the
 * Python package) links, loads or calls this code; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the
 * checker / CPU baseline.
 *
 * Parity status: the reference ships no tests, fixtures or golden vectors and
 * executing it in this pipeline was denied, so the
 * environment semantics are "parity unpinned" against reference outputs. The
 * CPython-random part IS pinned: tests/golden/mt_vectors.json was generated
 * from CPython's own stdlib. The environment semantics are cross-checked
 * against an object-faithful Python restatement (oracle/pyref.py) and against
 * hand-derived known-answer scenarios (tests/golden/kat_*.json).
 */
#ifndef MS_ORACLE_H
#define MS_ORACLE_H

#include <stdint.h>

#include "../include/marlsched.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mso_env mso_env;

typedef struct mso_step_out {
    /* rewards (Reward.py) */
    double* offer;        /* [N][L] offerNetRewards / coreChooserRewards */
    double* price;        /* [N][L] priceChooserRewards (free) */
    int64_t* acceptor;    /* [N][C] */
    int64_t* auctioneer;  /* [C] */
    int64_t* agent;       /* [N] */
    int64_t termination_revenue; /* env.terminationRevenues increment (fixed prices) */
    /* events */
    ms_accept_rec* accepted;   /* [C] by core */
    ms_term_rec* terminated;   /* [C] by core */
    /* acception quality (SchedulingEnvironment.py:174-192): per accepted
     * non-auctioneer offer, in execution order */
    double* quality;      /* [C] */
    int32_t n_quality;
} mso_step_out;

mso_env* mso_create(const ms_config* cfg, uint64_t seed);
void mso_destroy(mso_env* env);
int mso_shape(const mso_env* env, ms_shape* out);

/* world.step1 + observation gathering + getRewards. acc_act [N][C],
 * off_core [N][L], off_price [N][L] (free) or NULL, auct_act [C] or NULL
 * (NULL = HardcodedAuctioneerAcceptor on the env RNG, drawn before the step). */
int mso_step(mso_env* env, const int32_t* acc_act, const int32_t* off_core,
             const int32_t* off_price, const int32_t* auct_act, mso_step_out* out);

/* HardcodedAuctioneerAcceptor.selectAction for all cores (consumes RNG). */
void mso_auctioneer_actions(mso_env* env, int32_t* out);

/* Observations of the current state; ids are the correspondingOfferIDs. Any NULL skipped.
 * acc_obs [N][C][D_acc], acc_ids [N][C][O], off_obs [N][L][D_off],
 * auct_obs [C][D_acc], auct_ids [C][O]. */
void mso_observe(const mso_env* env, int32_t* acc_obs, int32_t* acc_ids, int32_t* off_obs,
                 int32_t* auct_obs, int32_t* auct_ids);

/* canonical state export/import (E = 1 views of ms_state_host) */
void mso_export(const mso_env* env, const ms_state_host* out);
int mso_import(mso_env* env, const ms_state_host* in);
int64_t mso_round(const mso_env* env);
uint32_t mso_flags(const mso_env* env);

/* CPython random restatement on the env stream (for tests) */
uint32_t mso_genrand(mso_env* env);
double mso_random(mso_env* env);
uint32_t mso_randbelow(mso_env* env, uint32_t n);

/* standalone CPython-compatible MT19937 (seed, then draw) for golden vectors */
void mso_mt_seed_words(uint64_t seed, uint32_t* state624, int32_t* index);

/* batched driver used as the CPU baseline: E envs stepped with the given
 * actions ([E][...] int8 like the device ABI); threads = OpenMP threads (0 = all) */
int mso_step_batch(mso_env** envs, int64_t n_envs, const int8_t* acc_act, const int8_t* off_core,
                   const int8_t* off_price, int8_t* acc_obs, int8_t* off_obs, int32_t acc_stride,
                   int32_t off_stride, float* offer_rew, float* price_rew, int32_t* acc_rew,
                   int threads);

#ifdef __cplusplus
}
#endif

#endif
