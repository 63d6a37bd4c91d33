/*
 * marlsched.h — C ABI of libmarlsched.so, the MI355X-native hot path of
 * lr40/marl-scheduling (per-round environment step + policy act + PPO returns).
 *
 * The boundary replaces the reference's Python surface (paths relative to
 * /root/reference/src):
 *   ms_env_create   <- World.__init__                     world.py:211-254
 *                      + Env.__init__ (agents/collections) SchedulingEnvironment.py:253-348
 *   ms_env_reset    <- SchedulingEnv.reset                SchedulingEnvironment.py:85-109
 *   ms_env_step     <- SchedulingEnv.step                 SchedulingEnvironment.py:32-83
 *                      (World.step1 world.py:295-334, gatherObservations Agent.py:148-300,
 *                       gatherDividedAuctioneerObservation Auctioneer.py:20-77,
 *                       Auctioneer.getAuctioneerAction Auctioneer.py:95-102 +
 *                       HardcodedAuctioneerAcceptor HardcodedModules.py:48-78,
 *                       getDividedFixedPricesReward Reward.py:146-212,
 *                       getDividedFreePricesReward Reward.py:6-89)
 *   ms_env_randbelow <- random.randint/_randbelow on the env's global stream
 *                      (Agent.py:718,725; SchedulingEnvironment.py:317-326)
 *   ms_policy_act   <- PPO.selectAction / ActorCritic.act  PPOmodules.py:53-63,114-125
 *   ms_discounted_returns, ms_unit_returns <- PPO.update return estimate  PPOmodules.py:128-137
 *
 * Conventions: plain pointers and sizes; every device pointer is a HIP device
 * allocation owned by the caller unless stated; all work is enqueued on the
 * caller's stream (hipStream_t passed as void*; NULL = default stream); a handle
 * is not thread-safe; no pointer is retained after a call returns.
 * Errors are return codes (0 = ok); ms_last_error() gives the message of the
 * last failing call on the calling thread. No exception crosses the ABI.
 */
#ifndef MARLSCHED_H
#define MARLSCHED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MS_ABI_VERSION 18

#define MS_MAX_KINDS 16
#define MS_MAX_AGENTS 64
#define MS_MAX_CORES 64
#define MS_MAX_COLLECTION 32
#define MS_MAX_OFFERS 126 /* O = N*L; acceptor actions [0, O] must fit int8 */

/* return codes */
#define MS_OK 0
#define MS_EINVAL 22      /* bad argument / shape / config */
#define MS_ENOMEM 12      /* device or host allocation failed */
#define MS_EHIP 1001      /* a HIP runtime call failed */
#define MS_EOVERFLOW 75   /* a fatal per-env error flag is set (see MS_FLAG_*) */

/* per-env error flags (ORed over envs by ms_env_flags; sticky in each env's record). All but
 * SPAWN_EDGE are "fatal": the reference raises there, so once a completed round has set one, the
 * next ms_env_step returns MS_EOVERFLOW without launching (the round that set it cannot report
 * it: a step is asynchronous; the check reads a host-coherent word the kernel sets, no sync).
 * SPAWN_EDGE marks a documented deviation (the build clamps where the reference raises
 * UnboundLocalError) and does not stop stepping. ms_env_import clears them. */
#define MS_FLAG_LIABILITY_OVERFLOW 0x01u /* a core's liability chain exceeded liability_cap */
#define MS_FLAG_BAD_ACTION 0x02u         /* acceptor action outside [0, O] (reference asserts, world.py:389,404) */
#define MS_FLAG_COLLECTION_FULL 0x04u    /* insertJob into a full collection (reference raises, world.py:133) */
#define MS_FLAG_SPAWN_EDGE 0x08u         /* u >= accProbabilities[-1]; clamped to last kind (Agent.py:53-56) */
#define MS_FLAG_RNG_WINDOW 0x10u         /* a round drew past the 3 MT blocks it can reach (> 1248 words) */
#define MS_FLAG_GUARD 0x20u              /* offer recipient != core owner at execution (world.py:266) */
#define MS_FATAL_FLAGS (MS_FLAG_LIABILITY_OVERFLOW | MS_FLAG_BAD_ACTION | MS_FLAG_COLLECTION_FULL | \
                        MS_FLAG_RNG_WINDOW | MS_FLAG_GUARD)

/* RNG modes */
#define MS_RNG_CPYTHON_MT19937 0 /* per-env MT19937 with CPython random.seed/random/_randbelow semantics */

typedef struct ms_config {
    int32_t n_agents;          /* numberOfAgents            world.py:215 */
    int32_t n_cores;           /* numberOfCores             world.py:216 */
    int32_t collection_length; /* collectionLength          world.py:225 */
    int32_t n_kinds;           /* len(possibleJobPriorities) */
    int32_t job_priority[MS_MAX_KINDS]; /* possibleJobPriorities world.py:218 */
    int32_t job_length[MS_MAX_KINDS];   /* possibleJobLengths    world.py:217 */
    /* world.accProbabilities (world.py:220-222): Python left-to-right float sums */
    double acc_probability[MS_MAX_KINDS];
    int32_t n_fix_prices;              /* len(fixPricesList); fixed-price mode needs >= n_kinds */
    int32_t fix_price[MS_MAX_KINDS];   /* listOfFixPrices world.py:214, indexed by job kind */
    int32_t free_prices;               /* world.freePrices world.py:212 */
    int32_t commercial_reward;         /* commercialFreePriceReward Reward.py:22,36 */
    double net_zero_offer_reward;      /* env.netZeroOfferReward SchedulingEnvironment.py:30 */
    int32_t new_jobs_per_round;        /* newJobsPerRoundPerAgent world.py:236 */
    int32_t reward_multiplier;         /* rewardMultiplier world.py:246 (integer in every driver) */
    int32_t episode_length;            /* episodeLength world.py:243 */
    int32_t liability_cap;             /* entries kept per core liability chain (0 -> 128) */
    int32_t rng_mode;                  /* MS_RNG_* */
    int32_t reserved[7];
} ms_config;

/* Derived shapes of a configuration (all byte strides are multiples of 4). */
typedef struct ms_shape {
    int32_t n_agents, n_cores, collection_length;
    int32_t max_offers;        /* O = N*L (world.py:227-229) */
    int32_t acc_obs_dim;       /* D_acc = 3 + 2*O (PPOmodules.py:237-238) */
    int32_t acc_obs_stride;    /* bytes per acceptor/auctioneer obs row (D_acc rounded up to 4) */
    int32_t off_obs_dim;       /* D_off = 2*C + 2 (PPOmodules.py:257) */
    int32_t off_obs_stride;    /* bytes per offer obs row (D_off rounded up to 4) */
    int32_t acc_actions;       /* A_acc = O + 1 (reject index O) */
    int32_t off_actions;       /* A_off = C + 1 */
    int32_t price_actions;     /* A_pc = max(priorities) + 1 (PPOmodules.py:295) */
    int32_t liability_cap;
    int64_t env_record_bytes;  /* packed per-env state record on the device */
} ms_shape;

/* Actions for one step of all E envs (device pointers). acceptor and offer_core both NULL = the
 * hard-coded agents of HardcodedFixPriceEnvironment (SchedulingEnvironment.py:439-456,
 * DividedHardcodedAgent Agent.py:622-641, HardcodedModules.py:16-45, 81-109) act in-kernel on the env
 * stream (fixed prices only), before the auctioneer. */
typedef struct ms_actions {
    const int8_t* acceptor;    /* [E][N][C] in [0, O]; O = reject (world.py:391-404) */
    const int8_t* offer_core;  /* [E][N][L] core action a: core a+1 if a < C else no offer (world.py:412,450) */
    const int8_t* offer_price; /* [E][N][L] free prices only (world.py:452); NULL in fixed-price mode */
    const int8_t* auctioneer;  /* [E][C] or NULL = in-kernel HardcodedAuctioneerAcceptor on the env RNG */
} ms_actions;

/* Observation outputs (device pointers; any may be NULL to skip). */
typedef struct ms_obs_out {
    int8_t* acceptor;   /* [E][N][C][acc_obs_stride]  Agent.py:167-212 (pad bytes zero) */
    int8_t* offer;      /* [E][N][L][off_obs_stride]  Agent.py:271-300 */
    int8_t* auctioneer; /* [E][C][acc_obs_stride]     Auctioneer.py:34-77 */
    /* Compact acceptor observations (the [E][N][C] acceptor rows regenerated on demand): core_rows[e][c]
     * is the acceptor row core c's owner sees ([1, prio, rem, offers to c in ID order, pads]), core_owner
     * [E][C] its ownerID. Acceptor row (a, c) equals core_rows[e][c] when core_owner[e][c] == a + 1 and
     * the constant [0, -1, -1, (-2, -2) * O] otherwise (Agent.py:167-212; see ms_regen_acceptor_rows). */
    int8_t* core_rows;  /* [E][C][acc_obs_stride] */
    int8_t* core_owner; /* [E][C] */
} ms_obs_out;

/* Reward outputs (device pointers; any may be NULL to skip). */
typedef struct ms_reward_out {
    float* offer;           /* [E][N][L] offerNetRewards (fixed) / coreChooserRewards (free) */
    float* price;           /* [E][N][L] priceChooserRewards (free prices only) */
    int32_t* acceptor;      /* [E][N][C] acceptorNetRewards */
    int32_t* auctioneer;    /* [E][C]    auctioneerReward */
    int32_t* agent;         /* [E][N]    agentReward */
    /* getAggregatedFixedPricesReward (Reward.py:92-143), for the aggregated agents:
     * offerRewards[a] = sum of prio1 over a's accepted offers; acceptorRewards[a] = the
     * rewards of a's terminating jobs minus what a pays along the liability chains (no
     * recipient credit, unlike the divided acceptor rewards). */
    int32_t* aggregated_offer;     /* [E][N] */
    int32_t* aggregated_acceptor;  /* [E][N] */
} ms_reward_out;

/* One executed offer (world.acceptedOffers entry), stored at its core's index. */
typedef struct ms_accept_rec {
    int8_t valid;     /* 1 if an offer was executed on this core this round */
    int8_t offerer;   /* offererID (1..N) */
    int8_t recipient; /* recipientID (0 = auctioneer) */
    int8_t slot;      /* queuePosition */
    int8_t price;     /* offeredReward */
    int8_t nec_time;  /* necessaryTime */
    int8_t prio;      /* prio1 */
    int8_t kind;      /* jobKind */
    int8_t order;     /* position in world.acceptedOffers (execution order) */
    int8_t pad[3];
    int32_t round;    /* world.round at execution */
} ms_accept_rec;

/* One job termination (jobTerminationInfo + verweilzeiten entry) at its core's index. */
typedef struct ms_term_rec {
    int8_t valid;     /* 1 if the core's job terminated this round */
    int8_t owner;     /* ownerID */
    int8_t prio;      /* Prioritaet */
    int8_t init_len;  /* Bedienzeit */
    int32_t dwell;    /* Verweilzeit = round - birthDate (world.py:350-357) */
} ms_term_rec;

/* Per-replica episode accumulators of the training driver's metrics (trainPPO.py:172-226,
 * trainDQN.py:187-259): every ms_env_step that is given them adds its round into the slot of the
 * round's episode. The caller reads a slot once its episode is done (world.round % episodeLength
 * == 0, SchedulingEnvironment.py:64-67) and zeroes it before the slot is reused. Updated with
 * no-return device atomics, one env per group of lanes, so the order per replica is fixed. */
typedef struct ms_env_metrics {
    int64_t acceptor_reward;     /* sum over rounds and units of acceptorNetRewards */
    int64_t offer_reward;        /* sum of offerNetRewards / coreChooserRewards (prio1, integers) */
    double price_reward;         /* sum of priceChooserRewards (free prices) */
    int64_t auctioneer_reward;   /* sum over rounds of sum(auctioneerReward) (trainPPO.py:183) */
    int64_t termination_revenue; /* env.terminationRevenues (Reward.py:193; fixed prices) */
    double quality_sum;          /* sum over rounds with an acception of the round's mean
                                    acception quality (SchedulingEnvironment.py:174-192) */
    int32_t quality_rounds;      /* rounds counted in quality_sum */
    int32_t acception_amount;    /* sum over rounds of the number of non-auctioneer acceptions */
    int32_t rounds;              /* rounds added */
    int32_t pad;
    int32_t price_sum[MS_MAX_KINDS];   /* offeredReward of accepted offers, by jobKind (trainPPO.py:172-174) */
    int32_t price_count[MS_MAX_KINDS];
    int32_t dwell_sum[MS_MAX_KINDS];   /* round - birthDate - 1 of terminated jobs, by kind (world.py:350-357) */
    int32_t dwell_count[MS_MAX_KINDS];
    int64_t agent_reward[MS_MAX_AGENTS]; /* sum of agentReward */
} ms_env_metrics;

typedef struct ms_event_out {
    ms_accept_rec* accepted; /* [E][C] or NULL */
    ms_term_rec* terminated; /* [E][C] or NULL */
    /* [E][4] device u64 or NULL: per wave of the launch, its start and end on the s_memrealtime
     * clock (100 MHz) at [b][0..1] and on the shader clock (s_memtime) at [b][2..3] (ABI 16; a wave steps
     * 64 / lanes_per_env envs, so the first ceil(E * lanes_per_env / 64) entries are written); min start
     * to max end is the launch's span, shader cycles over 100 MHz ticks its clock. Measurement only:
     * four plain stores per wave. */
    uint64_t* launch_span;
    /* [metrics_slots][E] or NULL: round r (world.round before the step) adds into slot
     * (r / episode_length) % metrics_slots */
    ms_env_metrics* metrics;
    int32_t metrics_slots;
} ms_event_out;

/* Host-side canonical state (export/import for parity tests and KAT scenarios).
 * Arrays are host memory, shaped as noted, int32 unless stated. */
typedef struct ms_state_host {
    int32_t* round;        /* [E] world.round */
    uint32_t* flags;       /* [E] MS_FLAG_* */
    int32_t* core_owner;   /* [E][C] ownerID (0 = auctioneer) */
    int32_t* core_kind;    /* [E][C] job kind, -1 = empty job */
    int32_t* core_rem;     /* [E][C] remainingLength (-1 if empty) */
    int32_t* core_birth;   /* [E][C] birthDate */
    int32_t* slot_kind;    /* [E][N][L] -1 = empty */
    int32_t* slot_rem;     /* [E][N][L] */
    int32_t* slot_wait;    /* [E][N][L] Job.wait */
    int32_t* slot_birth;   /* [E][N][L] */
    int32_t* offer_core;   /* [E][N][L] pending offer of this slot: core index, -1 = none */
    int32_t* offer_recip;  /* [E][N][L] recipientID */
    int32_t* offer_price;  /* [E][N][L] offeredReward */
    int32_t* liab_n;       /* [E][C] chain length */
    int32_t* liab;         /* [E][C][cap][5] {offerer, recipient, price, nec_time, round}, oldest first */
    uint32_t* mt;          /* [E][624] MT19937 state words */
    int32_t* mt_index;     /* [E] mti (0..624) */
} ms_state_host;

typedef struct ms_env ms_env;

/* Create E independent env replicas in the reference initial state
 * (world.py:247, Core.__init__ world.py:30-37, JobCollection world.py:118-121),
 * env e's RNG seeded as CPython random.seed(seed + e). */
int ms_env_create(const ms_config* cfg, int64_t n_envs, uint64_t seed, ms_env** out);
void ms_env_destroy(ms_env* env);
int ms_env_shape(const ms_env* env, ms_shape* out);
int ms_config_shape(const ms_config* cfg, ms_shape* out);

/* Observations of the current state, no state change (SchedulingEnvironment.py:85-109). */
int ms_env_reset(ms_env* env, const ms_obs_out* obs, void* stream);

/* One round for all E envs (SchedulingEnvironment.py:32-83). Rewards/events are
 * fully written (zeros where nothing happened). Returns MS_EOVERFLOW (and launches nothing)
 * once an earlier completed round has raised a fatal flag (MS_FATAL_FLAGS). */
int ms_env_step(ms_env* env, const ms_actions* act, const ms_obs_out* obs,
                const ms_reward_out* rew, const ms_event_out* ev, void* stream);

/* Host round counter (all replicas advance together). */
int64_t ms_env_round(const ms_env* env);

/* Synchronises the stream and returns the OR of all env flags in *flags (MS_OK either way). */
int ms_env_flags(ms_env* env, uint32_t* flags, void* stream);

/* CPython random._randbelow(n) drawn on env e's stream (n >= 1); synchronous. */
int ms_env_randbelow(ms_env* env, int64_t env_index, uint32_t n, uint32_t* out, void* stream);

/* Auctioneer.getAuctioneerAction (Auctioneer.py:95-102) for all E envs on the current state, as
 * trainPPO.py:162 calls it before env.step: writes actions [E][C] (O = reject) and consumes the
 * tie-break draws of each env's stream; pass the actions to ms_env_step afterwards. */
int ms_env_auctioneer(ms_env* env, int8_t* actions, void* stream);

/* Env e's CPython random state (random.getstate()/setstate(), Modules/_randommodule.c): the 624
 * MT19937 words and the index. Synchronous. Lets an E = 1 driver share the global `random`
 * module with the env as the reference does (world.py spawn, Auctioneer ties, Agent.py:718). */
int ms_env_get_rng(ms_env* env, int64_t env_index, uint32_t* words, int32_t* index, void* stream);
int ms_env_set_rng(ms_env* env, int64_t env_index, const uint32_t* words, int32_t index, void* stream);

/* Copy the full state to / from host arrays (synchronous). Import validates
 * the reference invariants the kernel relies on. */
int ms_env_export(ms_env* env, const ms_state_host* out, void* stream);
int ms_env_import(ms_env* env, const ms_state_host* in, void* stream);

/* ---- policy act: fused Linear-tanh-Linear-tanh-Linear-softmax + Categorical ----
 * Rows: obs[e][u][stride] int8 for e < n_envs, u < n_units. Unit u uses weight
 * group g = u / units_per_group (units_per_group * n_groups == n_units), i.e.
 * divided nets (units_per_group = 1), locally shared (= sub-units per agent),
 * globally shared (n_groups = 1). Weights are torch nn.Linear layouts, stacked
 * over groups: w1 [G][H][D], b1 [G][H], w2 [G][H][H], b2 [G][H], w3 [G][A][H], b3 [G][A].
 * Sampling: inverse CDF of the normalised probabilities (torch Categorical,
 * PPOmodules.py:55-61) with u = uniform (Philox2x32-10 keyed by seed and the offset's high
 * word, counter (row, offset)) or, when uniforms != NULL, the given per-row uniform in [0,1).
 * Outputs: action[e*n_units+u] int8, logprob f32 (log of clamped normalised prob). */
typedef struct ms_mlp_params {
    const float *w1, *b1, *w2, *b2, *w3, *b3;
    int32_t in_dim;    /* D */
    int32_t hidden;    /* H (<= 64) */
    int32_t n_actions; /* A (<= 128) */
    int32_t n_groups;  /* G */
    /* Optional (ABI 13): the act kernels' per-lane weight fragments and the common row's sampling
     * table, made by ms_act_prepare from these weights (NULL: each acting wave derives them). A
     * fragment block whose header does not match the call's shape is ignored. Rebuild it whenever
     * the weights change (like ms_price_table_build). Other entry points ignore the field. */
    const void* act_frag;
    /* ABI 16: the Philox row counter of this call's row r (= e * n_units + u) is row_base + r. A caller
     * stepping replicas [e0, e0 + E) of a larger set passes row_base = e0 * n_units, so every replica
     * draws the numbers it would draw in one call over the whole set (a rank's shard, a stream's part).
     * For the single-net acceptor rule (word (i >> 6) & 1 of item i's draw) this holds when
     * e0 * units_per_group is a multiple of 128. 0 for a standalone call; ignored outside acting. */
    int64_t row_base;
} ms_mlp_params;

/* Bytes of the act fragment block of net p acting on rows of obs_stride bytes. */
size_t ms_act_frag_bytes(const ms_mlp_params* p, int32_t obs_stride);

/* Writes the act fragment block (frag, ms_act_frag_bytes) for net p's current weights: each acting
 * lane's layer-1 weight terms (hi + mid + lo, exact), its layer-2/3 weights and pre-scaled biases,
 * and, with common_row != NULL, the common row's sampling table (ms_policy_act_common /
 * _compact / ms_act_round_free). Acting with the block is bit-identical to acting without it; a
 * rollout makes it once instead of every acting wave of every round deriving it
 * (PPOmodules.py:53-63 runs policy_old, fixed between two updates). */
int ms_act_prepare(const ms_mlp_params* p, const int8_t* common_row, int32_t obs_stride, void* frag, void* stream);

/* The Philox counter offset is offset + *offset_dev (offset_dev may be NULL); a
 * device-resident offset lets a captured HIP graph draw fresh numbers per replay. */
int ms_policy_act(const ms_mlp_params* p, const int8_t* obs, int32_t obs_stride,
                  int64_t n_envs, int32_t n_units, int32_t units_per_group,
                  uint64_t seed, uint64_t offset, const uint64_t* offset_dev, const float* uniforms,
                  int8_t* action, float* logprob, void* stream);

/* ms_policy_act where many observation rows equal one common row (device, obs_stride bytes):
 * the acceptor rows of cores an agent does not own are all [0, -1, -1, (-2, -2) * O, 0 pad]
 * (Agent.py:167-212). The common row's network output is computed once per wave and every row
 * equal to it is sampled from that table; outputs are bit-identical to ms_policy_act's. */
int ms_policy_act_common(const ms_mlp_params* p, const int8_t* obs, int32_t obs_stride,
                         int64_t n_envs, int32_t n_units, int32_t units_per_group, const int8_t* common_row,
                         uint64_t seed, uint64_t offset, const uint64_t* offset_dev, const float* uniforms,
                         int8_t* action, float* logprob, void* stream);

/* ms_policy_act_common on compact acceptor observations (ms_obs_out.core_rows / core_owner):
 * core_rows [E][C][obs_stride], core_owner [E][C]; unit u = a*C + c of replica e acts on core row
 * (e, c) when core_owner[e][c] == a + 1 and on common_row otherwise (Agent.py:167-212). Outputs are
 * bit-identical to ms_policy_act_common on the [E][N*C] rows those regenerate. */
int ms_policy_act_compact(const ms_mlp_params* p, const int8_t* core_rows, const int8_t* core_owner,
                          int32_t obs_stride, int64_t n_envs, int32_t n_units, int32_t units_per_group, int32_t n_cores,
                          const int8_t* common_row, uint64_t seed, uint64_t offset, const uint64_t* offset_dev,
                          const float* uniforms, int8_t* action, float* logprob, void* stream);

/* FreePriceOfferPPO.selectAction (PPOmodules.py:312-332) in one launch: the core
 * chooser acts on the offer observation (D_off = 2C+2); the price chooser acts on
 * price_state = [obs[2a], obs[2a+1], obs[2C], obs[2C+1]] or [-5,-5,-5,-5] when a == 0
 * (written to price_state [E][U][4]); env_price = -5 if a == 0 else the price action
 * (the offer price world.py:452 sees). uniforms: [2][E*U] (core, price) or NULL.
 * price_unit_stride: 0 = price_state / price_action / price_logprob in [E][U] rows; else >= E and
 * unit-major, row (e, u) at u * price_unit_stride + e (a rollout ring [U][T][E] with the round's
 * offset: the update reads one unit's rows of every replica contiguously). env_price stays [E][U]. */
int ms_offer_act_free(const ms_mlp_params* core_chooser, const ms_mlp_params* price_chooser,
                      const int8_t* obs, int32_t obs_stride, int64_t n_envs, int32_t n_units,
                      int32_t units_per_group, int32_t n_cores, uint64_t seed, uint64_t offset,
                      const uint64_t* offset_dev, const float* uniforms, int8_t* core_action,
                      float* core_logprob, int8_t* price_state, int8_t* price_action,
                      float* price_logprob, int8_t* env_price, int64_t price_unit_stride, void* stream);

/* The price chooser's sampling table (FreePriceOfferPPO's second net, PPOmodules.py:316-330): its
 * input is 4 bytes taking few values, so the forward of every tabulated input is computed once per
 * weight update and each acting row samples from its entry (bit-identical to computing it).
 *   digit [4][256] int16: key offset of byte value v at position p (index v + 128), -1 = not
 *                         tabulated (such a row's tile computes the net instead);
 *   rows  [n_keys][4] int8: the input of every key (key = sum of its bytes' offsets);
 *   table [G][n_keys][32*ceil(A/16) + 4] f32: running sums, log-probs, S, last nonzero action. */
typedef struct ms_price_table {
    const int16_t* digit;
    const int8_t* rows;
    int32_t n_keys;
    float* table;
} ms_price_table;
int ms_price_table_build(const ms_mlp_params* price_chooser, const ms_price_table* table, void* stream);

/* getActionForAllAgents of a free-price round (SchedulingEnvironment.py:150-172) in one launch:
 * ms_offer_act_free on off_obs (Philox offset off_offset) and ms_policy_act_compact on (core_rows,
 * core_owner) (offset acc_offset), same seed and offset_dev; outputs identical to the two calls.
 * The offer and acceptor waves share the CUs, so neither launch waits out its own latency alone.
 * price_table (optional, built for the current price-chooser weights): the price chooser samples
 * from it. price_chooser NULL (ABI 16): a fixed-price round (SchedulingEnvironment.py:150-172 with the
 * offer units' ActorCritic, PPOmodules.py:53-63): core_chooser is the offer net, core_action /
 * core_logprob its outputs, and price_state, price_action, price_logprob, env_price and price_table
 * must be NULL; outputs identical to ms_policy_act + ms_policy_act_compact. */
int ms_act_round_free(const ms_mlp_params* core_chooser, const ms_mlp_params* price_chooser, const int8_t* off_obs,
                      int32_t off_stride, int32_t off_units, int32_t off_units_per_group, const ms_mlp_params* acceptor,
                      const int8_t* core_rows, const int8_t* core_owner, int32_t acc_stride, int32_t acc_units,
                      int32_t acc_units_per_group, int32_t n_cores, const int8_t* common_row, int64_t n_envs,
                      uint64_t seed, uint64_t off_offset, uint64_t acc_offset, const uint64_t* offset_dev,
                      int8_t* core_action, float* core_logprob, int8_t* price_state, int8_t* price_action,
                      float* price_logprob, int8_t* env_price, int8_t* acc_action, float* acc_logprob,
                      const ms_price_table* price_table, int64_t price_unit_stride, void* stream);

/* The next round's getActionForAllAgents fused into the env round (ABI 16; SchedulingEnvironment.py:
 * 150-172 with PPOmodules.py:53-63): after the round's observations, the wave that stepped a replica
 * samples that replica's next actions from them (still in its LDS), so a round is one launch instead of
 * an act launch and an env launch. For fixed-price rounds with compact acceptor observations and one
 * offer net and one acceptor net (n_groups 1, globally shared), each net one 32-input k-step and <= 16
 * actions, and act fragments (ms_act_prepare; the acceptor's with the common row's table). Outputs are
 * those of ms_act_round_free(offer, NULL, ...) on the emitted observations, bit for bit: off_offset /
 * acc_offset are that call's offsets, and each net's row_base its Philox row base. */
typedef struct ms_fused_act {
    ms_mlp_params offer;      /* the offer units' net, act_frag for obs rows of off_obs_stride bytes */
    ms_mlp_params acceptor;   /* the acceptors' net, act_frag with the common row's table */
    const int8_t* common_row; /* [acc_obs_stride] the foreign acceptor row (ms_policy_act_compact's) */
    uint64_t seed, off_offset, acc_offset;
    const uint64_t* offset_dev; /* may be NULL */
    int8_t* off_action;       /* [E][N*L] */
    float* off_logprob;       /* [E][N*L] */
    int8_t* acc_action;       /* [E][N*C] */
    float* acc_logprob;       /* [E][N*C] */
} ms_fused_act;

/* ms_env_step followed by the fused acting of `next` (obs must hold core_rows / core_owner and offer).
 * MS_EINVAL when the shapes are not supported (the caller then steps and acts in two calls). */
int ms_env_step_act(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                    const ms_event_out* ev, const ms_fused_act* next, void* stream);

/* 1 when ms_env_step_act can run this env's rounds (fixed prices, the shapes above), else 0. */
int ms_env_step_act_supported(const ms_env* env);

/* Per-round byte strides of ms_env_rollout_act's arrays: round t uses each array given to it
 * advanced by t * stride bytes (0: the same array every round), and the acting after round t draws
 * with off_offset / acc_offset + t * offset_step. */
typedef struct ms_round_strides {
    int64_t acceptor_action, offer_action;            /* ms_actions acceptor / offer_core */
    int64_t core_rows, core_owner, offer_obs;         /* ms_obs_out */
    int64_t offer_reward, acceptor_reward, agent_reward, auctioneer_reward;  /* ms_reward_out */
    int64_t next_off_action, next_off_logprob, next_acc_action, next_acc_logprob;  /* ms_fused_act outputs */
    uint64_t offset_step;
} ms_round_strides;

/* n_rounds consecutive ms_env_step_act calls in one launch (trainPPO.py:160-167's loop body for
 * rounds t = 0 .. n_rounds - 1 of a fixed-price rollout, ring arrays advanced per round by `strides`):
 * each wave steps its replicas and samples their next actions round after round, reading back what it
 * wrote, with no launch between rounds. The acting after the last round runs only when
 * act_after_last != 0. ev->launch_span (optional) records the whole launch ([waves][4]). Outputs
 * are bit-identical to the n_rounds separate calls. Same requirements as ms_env_step_act, plus
 * no accepted / terminated event records and no price / aggregated reward outputs. */
int ms_env_rollout_act(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                       const ms_event_out* ev, const ms_fused_act* next, const ms_round_strides* strides,
                       int32_t n_rounds, int32_t act_after_last, void* stream);

/* ABI 17: the locally shared free-price rollout (BASELINE cfg3; LocallySharedPPO + FreePriceOfferPPO, DESIGN
 * §1) in one launch: every round's getActionForAllAgents (SchedulingEnvironment.py:150-172) fused after the env
 * round that built its observations. A workgroup steps 4 * N replicas (16 lanes each) and then acts for them
 * with one wave per agent: the agent's core chooser + price chooser (FreePriceOfferPPO.selectAction,
 * PPOmodules.py:312-332) on its L offer rows of every replica and its acceptor net (LocallySharedPPO.selectAction,
 * PPOmodules.py:532-543) on its C compact acceptor rows, from the rows still in the workgroup's LDS. Outputs are
 * those of ms_act_round_free(core_chooser, price_chooser, ..., acceptor, ...) on the emitted observations, bit for
 * bit: off_offset / acc_offset are that call's offsets, each net's row_base its Philox row base. */
typedef struct ms_fused_act_free {
    ms_mlp_params core_chooser;   /* N groups (one per agent, L units each); act_frag for off_obs_stride rows */
    ms_mlp_params price_chooser;  /* N groups, 4 -> A with A <= 16 */
    ms_mlp_params acceptor;       /* N groups (C units each); act_frag with the common row's table */
    const int8_t* common_row;     /* [acc_obs_stride] the foreign acceptor row */
    const ms_price_table* price_table; /* built for price_chooser's weights (ms_price_table_build) */
    uint64_t seed, off_offset, acc_offset;
    const uint64_t* offset_dev;   /* may be NULL */
    int8_t* core_action;          /* [E][N*L] */
    float* core_logprob;          /* [E][N*L] */
    int8_t* price_state;          /* [E][N*L][4] */
    int8_t* price_action;         /* [E][N*L] */
    float* price_logprob;         /* [E][N*L] */
    int8_t* env_price;            /* [E][N*L] the next round's offer_price actions (one buffer for every round) */
    int8_t* acc_action;           /* [E][N*C] */
    float* acc_logprob;           /* [E][N*C] */
    /* nonzero: leave the acceptor items of cores their agent does not own (the common row's, sampled from its
     * table; the env reads only the owner's acceptor action, world.py:391-404) to ms_env_rollout_fill_common,
     * which the caller runs later, e.g. on another stream beside other work; 0: the call runs it itself */
    int32_t defer_common;
    /* (ABI 18; both NULL: the owned items go straight into acc_action / acc_logprob) [E][C] the owned acceptor
     * items' outputs by core, item (e, owner - 1, c) at e * C + c: the rollout writes them here and the common fill
     * then writes every item of acc_action / acc_logprob, whole lines instead of one item in eight per round */
    int8_t* own_action;
    float* own_logprob;
} ms_fused_act_free;

/* Per-round byte strides of ms_env_rollout_act_free (as ms_round_strides, plus the price chooser's arrays). */
typedef struct ms_round_strides_free {
    int64_t acceptor_action, offer_action;                 /* ms_actions acceptor / offer_core (offer_price: 0) */
    int64_t core_rows, core_owner, offer_obs;              /* ms_obs_out */
    int64_t offer_reward, price_reward, acceptor_reward, agent_reward, auctioneer_reward; /* ms_reward_out */
    int64_t next_core_action, next_core_logprob, next_price_state, next_price_action, next_price_logprob;
    int64_t next_acc_action, next_acc_logprob;             /* ms_fused_act_free outputs */
    uint64_t offset_step;
    int64_t next_own_action, next_own_logprob;             /* (ABI 18) ms_fused_act_free own_action / own_logprob */
} ms_round_strides_free;

/* n_rounds rounds of a locally shared free-price rollout in one launch: round t steps the env with the
 * actions act->acceptor / offer_core advanced by t strides and act->offer_price (the next->env_price buffer the
 * acting refills), writes obs / rewards advanced by t strides, and then (t < n_rounds - 1, or act_after_last)
 * samples round t + 1's actions into next's outputs advanced by t strides, with offsets + t * offset_step.
 * Bit-identical to n_rounds pairs of ms_env_step + ms_act_round_free. Requires free prices, compact acceptor
 * observations (core_rows, core_owner, offer), no events or metrics or aggregated rewards,
 * ms_env_rollout_act_free_supported, N groups per net, act fragments for both nets and a price table.
 * Every ring must hold n_rounds slots at its stride (the kernel does not see the sizes). MS_EINVAL otherwise. */
int ms_env_rollout_act_free(ms_env* env, const ms_actions* act, const ms_obs_out* obs, const ms_reward_out* rew,
                            const ms_event_out* ev, const ms_fused_act_free* next, const ms_round_strides_free* strides,
                            int32_t n_rounds, int32_t act_after_last, void* stream);

/* The acceptor outputs of ms_env_rollout_act_free(..., next->defer_common = 1, ...) that the launch left: every
 * acting round's items (e, a, c) with core_owner[e][c] != a + 1, with the same obs, next and strides as that call
 * and next->offset_dev holding the value it held then (the Philox offsets of those rounds). On any stream ordered
 * after the rollout launch and before the outputs are read. */
int ms_env_rollout_fill_common(const ms_env* env, const ms_obs_out* obs, const ms_fused_act_free* next,
                               const ms_round_strides_free* strides, int32_t n_rounds, int32_t act_after_last,
                               void* stream);

/* 1 when ms_env_rollout_act_free can run this env's rounds (free prices, N <= 8, max(N, C) <= 16, offer rows
 * <= 32 bytes with <= 16 core actions, acceptor rows of 33..64 bytes with 17..32 actions), else 0. */
int ms_env_rollout_act_free_supported(const ms_env* env);

/* Discounted Monte-Carlo returns + per-sequence normalisation (PPOmodules.py:128-137):
 * rewards [T][M] (f32, as stored per round), for each sequence m:
 * G_t = r_t + gamma*G_{t+1} in float64, cast to f32, then
 * (G - mean) / (std_unbiased + 1e-7); out [M][T] f32. */
int ms_discounted_returns(const float* rewards, int32_t T, int64_t M, int64_t row_stride,
                          double gamma, float* out, void* stream);

/* The same returns for the sub-unit each group trains on, read straight from the rollout
 * reward buffer: rewards [T][E][U] (f32, or int32 with rewards_i32 = 1), sequence (e, g) is
 * unit unit_of_group[g] of replica e; out [T][E][G] f32 (the ms_ppo_batch.returns layout).
 * unit_of_group may list the sub-units of several update draws (Agent.py:716-728) back to back:
 * draw d then reads returns + d*G_draw with returns_ld = G. */
int ms_unit_returns(const void* rewards, int32_t rewards_i32, int32_t T, int64_t E, int32_t U,
                    const int32_t* unit_of_group, int32_t G, double gamma, float* out, void* stream);

/* ---- fused PPO loss gradient (one K-epoch step of PPO.update, PPOmodules.py:144-168) ----
 * For every group g: d/dθ_g of
 *   mean_r[-min(ratio*adv, clamp(ratio, 1-eps, 1+eps)*adv)] + 0.5*mean_r[(V-G)^2] - 0.01*mean_r[entropy]
 * over the R = T*E transitions of sub-unit unit_of_group[g], read straight from the
 * int8 rollout buffer (row r = t*E + e). Gradients are written (not accumulated) in
 * torch .grad layouts; the optimizer step stays with the caller. Deterministic. */
typedef struct ms_ppo_batch {
    const int8_t* states;          /* [R][U][stride] observation rows */
    const int8_t* actions;         /* [R][U] */
    const float* old_logprobs;     /* [R][U] */
    const float* returns;          /* [T][E][G] normalised (ms_unit_returns output) */
    const int32_t* unit_of_group;  /* [G] device array */
    int32_t stride, T, U;
    int64_t E;
    /* optional [stride] device row: rows equal to it (the acceptor rows of cores an agent does not
     * own, Agent.py:167-212) share one forward pass, and their summed loss derivatives run through
     * one backward pass (the gradient is linear in them); NULL = every row on its own */
    const int8_t* common_row;
    /* row pitch of returns in floats (0 = the number of groups): returns[(t*E + e)*ld + g] */
    int32_t returns_ld;
    /* compact acceptor observations (with common_row): states = core rows [R][n_cores][stride] and
     * core_owner [R][n_cores] (ms_obs_out.core_rows / core_owner per round); unit u = a*C + c of row r
     * reads core row (r, c) when core_owner[r][c] == a + 1, else common_row. NULL: states [R][U][stride] */
    const int8_t* core_owner;
    int32_t n_cores;
    /* 0: rows of 4 bytes (stride 4, nets of <= 4 inputs and <= 32 actions, no common_row) are keyed:
     * each group's distinct rows get one forward and one backward pass, and each row adds its loss
     * derivatives to its distinct row's int64 fixed-point sums (2^-20); -1: every row on its own */
    int32_t row_keys;
    /* 0: states [R][U][stride], actions / old_logprobs [R][U]; else >= R and unit-major: row (r, u) at
     * u * unit_stride + r in all three (e.g. [U][T][E] rollout rings; not with core_owner) */
    int64_t unit_stride;
} ms_ppo_batch;

typedef struct ms_ppo_grads {  /* device outputs, [G][...] like the weights */
    float *w1, *b1, *w2, *b2, *w3, *b3;       /* actor */
    float *cw1, *cb1, *cw2, *cb2, *cw3, *cb3; /* critic (output width 1) */
    float* loss;                              /* [G][3]: mean(-min(surr)), mean((V-G)^2), mean(entropy) */
} ms_ppo_grads;

size_t ms_ppo_workspace_bytes(const ms_mlp_params* actor, int64_t rows);
int ms_ppo_grad(const ms_mlp_params* actor, const ms_mlp_params* critic, const ms_ppo_batch* batch, float eps_clip,
                void* workspace, size_t workspace_bytes, const ms_ppo_grads* grads, void* stream);

/* ---- aggregated agents (AggregatedAgent Agent.py:73-140, AggregatedFixPricePPOAgent :359-391,
 * FullyAggregatedFixPricePPOAgent :393-492) around ms_env_step ----
 * Observations from the divided rows ms_env_step / ms_env_reset wrote (acc_obs
 * [E][N][C][acc_obs_stride], off_obs [E][N][L][off_obs_stride]); any output may be NULL:
 *   agg_acceptor [E][N][align4(C*D_acc)]        concat over cores of the acceptor rows (Agent.py:82-124)
 *   agg_offer    [E][N][align4(2C+2L)]          cores' (prio, rem), then slots' (prio, rem) (Agent.py:126-134)
 *   fully        [E][N][align4(2C+2L+C*D_acc)]  concat(offer, acceptor) (Agent.py:464)
 * Pad bytes are zero. */
int ms_aggregate_obs(const ms_config* cfg, int64_t n_envs, const int8_t* acc_obs, const int8_t* off_obs,
                     int8_t* agg_acceptor, int8_t* agg_offer, int8_t* fully, void* stream);
/* Agent action numbers -> the divided actions ms_env_step takes (numberToNDimensionalAction
 * Agent.py:644-666: action of core c = digit c of the acceptor number in base O+1, of slot s =
 * digit s of the offer number in base C+1). fully = 0: actions = acceptor numbers [E][N] then
 * offer numbers [E][N]; fully = 1: actions [E][N], acceptor = a / (C+1)^L, offer = a % (C+1)^L
 * (Agent.py:469-473). Out-of-range numbers (ValueError in the reference) decode as "reject all /
 * offer nothing" and are counted into *n_bad (device int32, may be NULL). EINVAL when the
 * action space exceeds int32. */
int ms_decode_aggregated(const ms_config* cfg, int64_t n_envs, const int32_t* actions, int32_t fully,
                         int8_t* acceptor, int8_t* offer_core, int32_t* n_bad, void* stream);

/* The aggregated agents' nets (AggregatedAcceptorPPO / AggregatedOfferPPO, PPOmodules.py:177-210,
 * 32 hidden units; FullyAggregatedPPO :213-232, 64): ActorCritic of hidden width 32 or 64, in_dim
 * 1..255, n_actions 1..2^24, one net per group (agent). Replace ActorCritic.act's torch forward +
 * Categorical.sample (PPOmodules.py:53-63, called by PPO.selectAction :114-125) and the autograd
 * of PPO.update (:127-174).
 *
 * ms_wide_act: rows (e, g) of obs [n_rows][G][obs_stride] int8 (obs_stride >= in_dim, multiple of
 * 4) through group g's actor; the action is the inverse-CDF sample at uniforms[e][g] (the number of
 * running sums of exp(z - max) that stay <= u * S) and logprob its log(clamp(p, eps, 1 - eps)).
 * action / logprob [n_rows][G]. */
int ms_wide_act(const ms_mlp_params* actor, const int8_t* obs, int32_t obs_stride, int64_t n_rows,
                const float* uniforms, int32_t* action, float* logprob, void* stream);

typedef struct ms_wide_batch {
    const int8_t* states;      /* row r of group g at states + (r * G + g) * stride (the [T][E][N] rings, r = t*E + e) */
    const int32_t* actions;    /* [R][G] */
    const float* old_logprob;  /* [R][G] */
    const float* returns;      /* [G][R] normalised */
    int32_t stride;            /* >= in_dim, multiple of 4 */
    int64_t rows;              /* R */
} ms_wide_batch;

/* One K-epoch gradient of PPO.update for the wide nets: grads = d/dθ of each group's
 * mean_r[-min(surr)] + 0.5 mean_r[(V-G)^2] - 0.01 mean_r[entropy] (same outputs as ms_ppo_grad;
 * the tensors are overwritten). Deterministic (fixed-order sums). */
size_t ms_wide_workspace_bytes(const ms_mlp_params* actor, int64_t rows);
int ms_wide_grad(const ms_mlp_params* actor, const ms_mlp_params* critic, const ms_wide_batch* batch, float eps_clip,
                 void* workspace, size_t workspace_bytes, const ms_ppo_grads* grads, void* stream);

/* Agent rows regenerated from compact observations (ms_obs_out.core_rows / core_owner, kept per
 * record in a replay memory of M records): for b < n_rows, record frame[b] seen by agent agent[b]
 * (0-based):
 *   acceptor [n_rows][align4(C * D_acc)]  the aggregated acceptor row (Agent.py:82-124): concat over
 *            cores c of core_rows[m][c][0:D_acc] if core_owner[m][c] == agent + 1, else the foreign
 *            row [0, -1, -1, (-2, -2) * O];
 *   offer    [n_rows][align4(2C + 2L)]    the aggregated offer row (Agent.py:126-134): the cores'
 *            (prio, rem) = core_rows[m][c][1:3], then slot_pairs[m][agent][s][0:2] ([M][N][L][2]).
 * Either output may be NULL; pad bytes are zero. */
int ms_regen_agent_rows(const ms_config* cfg, const int8_t* core_rows, const int8_t* core_owner,
                        const int8_t* slot_pairs, const int64_t* frame, const int32_t* agent, int64_t n_rows,
                        int8_t* acceptor, int8_t* offer, void* stream);

/* ---- Adam step (torch.optim.Adam as PPO.__init__ builds it, PPOmodules.py:100-112) ----
 * One optimizer.step() over the tensors of one PPO group: tensor i uses lr[lr_group[i]] (actor
 * and critic parameter groups), betas (beta1, beta2), eps, no weight decay, bias corrections of
 * step `step` (1-based, the value of torch's state["step"] after its increment). Updates param,
 * exp_avg and exp_avg_sq in place, in f32 (torch's foreach formula; the scalars are rounded
 * to f32 as torch passes them). At most MS_ADAM_MAX_TENSORS tensors per call. */
#define MS_ADAM_MAX_TENSORS 16
typedef struct ms_adam_tensor {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
    int32_t lr_group;
} ms_adam_tensor;
int ms_adam_step(const ms_adam_tensor* tensors, int32_t n_tensors, const double* lr, int32_t n_lr, int64_t step,
                 double beta1, double beta2, double eps, void* stream);
/* ms_adam_step with the step count read from device memory (*step_dev, >= 1, advanced by the
 * caller before each step): a captured HIP graph replays it with the current count. */
int ms_adam_step_dev(const ms_adam_tensor* tensors, int32_t n_tensors, const double* lr, int32_t n_lr,
                     const int64_t* step_dev, double beta1, double beta2, double eps, void* stream);

/* ---- DQN units: DQNEntity (DQNmodules.py:34-94) and optimize_model (DQNmodules.py:97-154) for the
 * DQN env (DQNDividedFixedPricesEnv SchedulingEnvironment.py:351-436, DividedFixPriceDQNAgent
 * Agent.py:303-356), G nets of one unit type batched over groups and replicas ----
 * Nets: nn.Sequential(Linear(D, 16), Tanh, Linear(16, A)), stacked over groups (nn.Linear layouts). */
typedef struct ms_qnet_params {
    const float *w1, *b1, *w2, *b2; /* [G][16][D], [G][16], [G][A][16], [G][A] */
    int32_t in_dim;                 /* D (<= 256) */
    int32_t hidden;                 /* must be 16 */
    int32_t n_actions;              /* A (<= 127) */
    int32_t n_groups;               /* G */
} ms_qnet_params;

/* selectAction (DQNmodules.py:56-70) for rows obs[e][u][stride] (unit u uses group
 * u / units_per_group): greedy[e*U+u] = the first argmax of Q; action = greedy when the row's first
 * uniform u1 > eps_threshold (RUN_END + (RUN_START - RUN_END) * exp(-round / RUN_DECAY)), else
 * floor(u2 * A) (random.randrange). uniforms: [2][E*U] doubles in [0, 1) or NULL = Philox4x32-10
 * keyed by seed, counter (row, offset + *offset_dev). greedy may be NULL. */
int ms_dqn_act(const ms_qnet_params* q, const int8_t* obs, int32_t obs_stride, int64_t n_envs, int32_t n_units,
               int32_t units_per_group, double eps_threshold, const double* uniforms, uint64_t seed, uint64_t offset,
               const uint64_t* offset_dev, int8_t* action, int8_t* greedy, void* stream);

/* A minibatch of every group: the replay memories of all (replica, unit) pairs, [E][U][capacity] transitions
 * (ReplayMemory DQNmodules.py:13-31, Transition(state, action, next_state, reward)), and for each pair
 * `batch` sampled memory indices (np.random.choice(memory[:nextFreeIndex], BATCH_SIZE) in the reference). */
typedef struct ms_dqn_batch {
    const int8_t* states;      /* [E][U][capacity][stride] */
    const int8_t* next_states; /* [E][U][capacity][stride] */
    const int8_t* actions;     /* [E][U][capacity] */
    const float* rewards;      /* [E][U][capacity] */
    const int32_t* samples;    /* [E][U][batch], each in [0, capacity) */
    int32_t stride, n_units, units_per_group, capacity, batch;
    int64_t n_envs;
    float gamma;               /* GAMMA of the unit type (OFFER_GAMMA / ACCEPTOR_GAMMA) */
} ms_dqn_batch;

typedef struct ms_qnet_grads { /* device outputs [G][...] like the weights */
    float *w1, *b1, *w2, *b2;
    float* loss;               /* [G] SmoothL1 loss, mean over the group's rows */
} ms_qnet_grads;

/* Gradient of mean SmoothL1(Q(s)[a], r + gamma * max Q_target(s')) over each group's
 * units_per_group * E * batch rows (one minibatch per replica: the replicas' mean loss), written
 * clamped to [-grad_clip, grad_clip] (grad_clip <= 0: none); the Adam step is ms_adam_step.
 * Deterministic (fixed summation order). */
size_t ms_dqn_workspace_bytes(const ms_qnet_params* q, int64_t rows_per_group);
int ms_dqn_grad(const ms_qnet_params* policy, const ms_qnet_params* target, const ms_dqn_batch* batch, float grad_clip,
                void* workspace, size_t workspace_bytes, const ms_qnet_grads* grads, void* stream);

/* ---- Branching DQN acting (BranchingDQNModules.py:75-123), BASELINE cfg5 ----
 * One BranchingQNetwork (Linear(obs,128)-ReLU-Linear(128,128)-ReLU, value head, ac_dim advantage
 * heads of n actions) with its heads stacked: head b = rows b*n .. b*n+n-1 of wa / ba. */
typedef struct ms_bdqn_params {
    const float *w1, *b1;   /* [128][obs], [128] */
    const float *w2, *b2;   /* [128][128], [128] */
    const float *wv, *bv;   /* [1][128], [1] */
    const float *wa, *ba;   /* [ac_dim*n][128], [ac_dim*n] */
    int32_t obs, ac_dim, n; /* n <= 128, ac_dim <= 127 */
} ms_bdqn_params;

/* Bytes of the prepared layer 1 (three exact bf16 terms of W1 over `segs` input segments of `seg`
 * values, each padded to a multiple of 32; then the segments' products W1_c F, segs x 128 floats). */
size_t ms_bdqn_workspace_bytes(int32_t seg, int32_t segs);

/* Prepares W1 for ms_bdqn_layer1_compact / ms_bdqn_act (once per weight change; seg * segs must be
 * obs). With base != NULL also writes W1_c F of every segment c into the workspace and
 * base[128] = b1 + sum_c W1_c F (in segment order), F the foreign acceptor row of
 * seg = D_acc values [0, -1, -1, (-2, -2) * O] (Agent.py:167-212). */
int ms_bdqn_prepare(const ms_bdqn_params* q, int32_t seg, int32_t segs, void* workspace, size_t workspace_bytes,
                    float* base, void* stream);

/* Scratch bytes of ms_bdqn_layer1_compact / ms_bdqn_act_compact: n_envs * n_cores * 128 floats of
 * per-(replica, core) layer-1 products, then (act_compact) the owning-agent masks and row list. */
size_t ms_bdqn_layer1_scratch_bytes(int64_t n_envs, int32_t n_cores);

/* Layer-1 pre-activations of every agent's aggregated acceptor row (Agent.py:82-124: its C acceptor
 * rows in core order, row c = core_rows[e][c] if core_owner[e][c] == a + 1 else F) from the compact
 * observations: h1 [n_envs * n_agents][128], row e * n_agents + a. workspace / base from
 * ms_bdqn_prepare(seg = acc_dim, segs = n_cores); scratch of ms_bdqn_layer1_scratch_bytes.
 * Deterministic. */
int ms_bdqn_layer1_compact(const ms_bdqn_params* q, const void* workspace, const float* base, const int8_t* core_rows,
                           const int8_t* core_owner, int64_t n_envs, int32_t n_agents, int32_t n_cores,
                           int32_t acc_dim, int32_t acc_stride, void* scratch, size_t scratch_bytes, float* h1,
                           void* stream);

/* get_action (BranchingDQNModules.py:117-123), epsilon-greedy per row (:181-186): a row with
 * explore[r] != 0 takes rand_action[r][*]; the others take, per branch, the first maximum of
 * q = (value + adv) - mean(adv) (:98). Layer 1 from h1 [n_rows][128] (pre-activations), or with
 * h1 == NULL from int8 rows x [n_rows][x_stride] and workspace = ms_bdqn_prepare(seg = obs,
 * segs = 1). explore may be NULL (all greedy). action: [n_rows][ac_dim] int8. */
int ms_bdqn_act(const ms_bdqn_params* q, const float* h1, const int8_t* x, int32_t x_stride, const void* workspace,
                int64_t n_rows, const uint8_t* explore, const int8_t* rand_action, int8_t* action, void* stream);

/* ms_bdqn_layer1_compact + ms_bdqn_act without the h1 rows: the P rows of every (replica, core) go to
 * scratch and the act kernel adds an agent's owned cores' rows to base itself (the same sum in the
 * same order, so the actions equal those of ms_bdqn_act on ms_bdqn_layer1_compact's h1). Only the
 * rows of agents that own a core run through the heads; an agent owning none has layer 1 = base, and
 * all of those take the greedy actions of that one common row (or their random ones where explored).
 * Rows e * n_agents + a, n_agents <= 64; arguments as those two functions'. */
int ms_bdqn_act_compact(const ms_bdqn_params* q, const void* workspace, const float* base, const int8_t* core_rows,
                        const int8_t* core_owner, int64_t n_envs, int32_t n_agents, int32_t n_cores, int32_t acc_dim,
                        int32_t acc_stride, void* scratch, size_t scratch_bytes, const uint8_t* explore,
                        const int8_t* rand_action, int8_t* action, void* stream);

/* ---- Branching DQN update (BranchingDQN.update_policy, BranchingDQNModules.py:125-164) ----
 * One role's minibatch of `batch` (<= 128) transitions: int8 observation rows of the states and
 * next states ([batch][ld]), the taken action of every branch ([batch][actions_ld] int8), rewards
 * and masks (0 at an episode end) [batch] f32. */
typedef struct ms_bdqn_batch {
    const int8_t* states;
    const int8_t* next_states;
    int32_t ld;
    const int8_t* actions;
    int32_t actions_ld;
    const float* rewards;
    const float* masks;
    int32_t batch;
} ms_bdqn_batch;

/* The online net's gradient tensors (the layout of ms_bdqn_params) and the loss [1]. */
typedef struct ms_bdqn_grads {
    float *w1, *b1, *w2, *b2, *wv, *bv, *wa, *ba;
    float* loss;
} ms_bdqn_grads;

size_t ms_bdqn_update_workspace_bytes(const ms_bdqn_params* q, int32_t batch);

/* The gradient of update_policy on one minibatch: current = q(s) at the taken actions (:135),
 * argmax = the first maximum of q(s') per branch, max_next = mean over the branches of target(s') at
 * argmax (:139-142), expected = r + max_next * gamma * mask (:144), loss = mse_loss(expected, current)
 * over [batch, ac_dim] (:145), every gradient element clamped to [-grad_clip, grad_clip] (:157-158;
 * grad_clip <= 0: no clamp, as ms_dqn_grad)
 * and written to grads (the Adam step is ms_adam_step / ms_adam_step_dev). Deterministic. */
int ms_bdqn_update(const ms_bdqn_params* q, const ms_bdqn_params* target, const ms_bdqn_batch* batch, float gamma,
                   float grad_clip, void* workspace, size_t workspace_bytes, const ms_bdqn_grads* grads, void* stream);

const char* ms_last_error(void);
int ms_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MARLSCHED_H */
