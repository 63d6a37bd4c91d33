/*
 * ms_oracle.c — CPU restatement of the marl-scheduling per-round step.
 *
 * TEST INFRASTRUCTURE ONLY (see ms_oracle.h): the checker for the HIP path and
 * the CPU baseline of bench.py. Written object-by-object after the reference
 * (paths relative to /root/reference/src); every function cites what it follows.
 * Compile without -ffast-math: settlement depends on IEEE double division and
 * round-half-even (Reward.py:200-201).
 */
#include "ms_oracle.h"

#include <fenv.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* CPython random (Modules/_randommodule.c, Lib/random.py:239-249,366,480-494) */

#define MT_N 624
#define MT_M 397

typedef struct {
    uint32_t mt[MT_N];
    int mti;
} mso_mt;

static void mt_init_genrand(mso_mt* r, uint32_t s) {
    r->mt[0] = s;
    for (int i = 1; i < MT_N; i++)
        r->mt[i] = 1812433253u * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint32_t)i;
    r->mti = MT_N;
}

static void mt_init_by_array(mso_mt* r, const uint32_t* key, int len) {
    mt_init_genrand(r, 19650218u);
    int i = 1, j = 0;
    int k = MT_N > len ? MT_N : len;
    for (; k; k--) {
        r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++;
        j++;
        if (i >= MT_N) {
            r->mt[0] = r->mt[MT_N - 1];
            i = 1;
        }
        if (j >= len) j = 0;
    }
    for (k = MT_N - 1; k; k--) {
        r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= MT_N) {
            r->mt[0] = r->mt[MT_N - 1];
            i = 1;
        }
    }
    r->mt[0] = 0x80000000u;
}

/* random.seed(int): key = 32-bit little-endian chunks of abs(seed), >= 1 word */
static void mt_seed(mso_mt* r, uint64_t seed) {
    uint32_t key[2];
    int len = 1;
    key[0] = (uint32_t)seed;
    key[1] = (uint32_t)(seed >> 32);
    if (key[1]) len = 2;
    mt_init_by_array(r, key, len);
}

static void mt_twist(mso_mt* r) {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    uint32_t y;
    int kk;
    for (kk = 0; kk < MT_N - MT_M; kk++) {
        y = (r->mt[kk] & 0x80000000u) | (r->mt[kk + 1] & 0x7fffffffu);
        r->mt[kk] = r->mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < MT_N - 1; kk++) {
        y = (r->mt[kk] & 0x80000000u) | (r->mt[kk + 1] & 0x7fffffffu);
        r->mt[kk] = r->mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (r->mt[MT_N - 1] & 0x80000000u) | (r->mt[0] & 0x7fffffffu);
    r->mt[MT_N - 1] = r->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    r->mti = 0;
}

static uint32_t mt_genrand(mso_mt* r) {
    if (r->mti >= MT_N) mt_twist(r);
    uint32_t y = r->mt[r->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

static double mt_random(mso_mt* r) {
    uint32_t a = mt_genrand(r) >> 5, b = mt_genrand(r) >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

static int bit_length(uint32_t n) {
    int k = 0;
    while (n) {
        k++;
        n >>= 1;
    }
    return k;
}

/* Random._randbelow_with_getrandbits (random.py:239-249); getrandbits(k<=32) = genrand >> (32-k) */
static uint32_t mt_randbelow(mso_mt* r, uint32_t n) {
    if (!n) return 0;
    int k = bit_length(n);
    uint32_t v = mt_genrand(r) >> (32 - k);
    while (v >= n) v = mt_genrand(r) >> (32 - k);
    return v;
}

void mso_mt_seed_words(uint64_t seed, uint32_t* state624, int32_t* index) {
    mso_mt r;
    mt_seed(&r, seed);
    memcpy(state624, r.mt, sizeof(r.mt));
    *index = r.mti;
}

/* ------------------------------------------------------------------------- */
/* World objects (world.py:27-207) */

typedef struct {
    int empty;   /* Job.empty */
    int kind;    /* jobKind (-1 empty) */
    int prio;    /* priority (-1 empty) */
    int rem;     /* remainingLength (-1 empty) */
    int init_len;
    int birth;   /* birthDate */
    int wait;    /* Job.wait */
} mso_job;

typedef struct {
    int offer_id, offerer, recipient, core_id, queue_pos, price, nec_time, prio1, kind, round;
} mso_offer;

struct mso_env {
    ms_config cfg;
    int N, C, L, O, cap;
    /* cores (Core, world.py:27-76): 1-based ids = index + 1 */
    mso_job* core_job;
    int* core_owner;
    /* agents' collections (JobCollection world.py:117-141) */
    mso_job* coll;    /* [N][L] */
    int* free_slots;  /* numberOfFreeSlots [N] */
    /* world.offers, in creation (= offerID) order */
    mso_offer* offers;
    int n_offers;
    /* liabilityList[core] (world.py:238): stored oldest first, iterated newest first */
    mso_offer* liab;  /* [C][cap] */
    int* liab_n;
    /* formerCorePrios / formerCoreLengths (SchedulingEnvironment.py:24-25,70-71) */
    int* former_prio;
    int* former_len;
    int round;
    uint32_t flags;
    mso_mt rng;
};

static mso_job empty_job(void) {
    mso_job j;
    j.empty = 1;
    j.kind = -1;
    j.prio = -1;
    j.rem = -1;
    j.init_len = -1;
    j.birth = -1;
    j.wait = 0;
    return j;
}

mso_env* mso_create(const ms_config* cfg, uint64_t seed) {
    if (cfg->n_agents < 1 || cfg->n_cores < 1 || cfg->collection_length < 1 || cfg->n_kinds < 1 ||
        cfg->n_kinds > MS_MAX_KINDS)
        return NULL;
    mso_env* e = (mso_env*)calloc(1, sizeof(mso_env));
    e->cfg = *cfg;
    e->N = cfg->n_agents;
    e->C = cfg->n_cores;
    e->L = cfg->collection_length;
    e->O = e->N * e->L; /* maxAmountOfOffersToOneAgent world.py:227-229 */
    e->cap = cfg->liability_cap > 0 ? cfg->liability_cap : 128;
    e->core_job = (mso_job*)calloc(e->C, sizeof(mso_job));
    e->core_owner = (int*)calloc(e->C, sizeof(int));
    e->coll = (mso_job*)calloc((size_t)e->N * e->L, sizeof(mso_job));
    e->free_slots = (int*)calloc(e->N, sizeof(int));
    e->offers = (mso_offer*)calloc((size_t)e->N * e->L, sizeof(mso_offer));
    e->liab = (mso_offer*)calloc((size_t)e->C * e->cap, sizeof(mso_offer));
    e->liab_n = (int*)calloc(e->C, sizeof(int));
    e->former_prio = (int*)calloc(e->C, sizeof(int));
    e->former_len = (int*)calloc(e->C, sizeof(int));
    for (int c = 0; c < e->C; c++) {
        e->core_job[c] = empty_job(); /* Core.__init__ world.py:35-37 */
        e->core_owner[c] = 0;
        e->former_prio[c] = -1;
        e->former_len[c] = -1;
    }
    for (int i = 0; i < e->N * e->L; i++) e->coll[i] = empty_job(); /* world.py:119 */
    for (int a = 0; a < e->N; a++) e->free_slots[a] = e->L;
    e->round = 0;
    mt_seed(&e->rng, seed);
    return e;
}

void mso_destroy(mso_env* e) {
    if (!e) return;
    free(e->core_job);
    free(e->core_owner);
    free(e->coll);
    free(e->free_slots);
    free(e->offers);
    free(e->liab);
    free(e->liab_n);
    free(e->former_prio);
    free(e->former_len);
    free(e);
}

/* same arithmetic as the product's ms_config_shape, restated so that the
 * oracle neither links nor exports product symbols */
int mso_shape(const mso_env* e, ms_shape* s) {
    const ms_config* cfg = &e->cfg;
    memset(s, 0, sizeof(*s));
    s->n_agents = cfg->n_agents;
    s->n_cores = cfg->n_cores;
    s->collection_length = cfg->collection_length;
    s->max_offers = cfg->n_agents * cfg->collection_length;
    s->acc_obs_dim = 3 + 2 * s->max_offers;
    s->acc_obs_stride = (s->acc_obs_dim + 3) & ~3;
    s->off_obs_dim = 2 * cfg->n_cores + 2;
    s->off_obs_stride = (s->off_obs_dim + 3) & ~3;
    s->acc_actions = s->max_offers + 1;
    s->off_actions = cfg->n_cores + 1;
    int mp = cfg->job_priority[0];
    for (int i = 1; i < cfg->n_kinds; i++)
        if (cfg->job_priority[i] > mp) mp = cfg->job_priority[i];
    s->price_actions = mp + 1; /* world.maxSumToOffer + 1, PPOmodules.py:295 */
    s->liability_cap = cfg->liability_cap > 0 ? cfg->liability_cap : 128;
    s->env_record_bytes = 0;
    return 0;
}

/* Agent.updateOwnedCores (Agent.py:35-36): len(ownedCores) */
static int owned_cores(const mso_env* e, int agent_id) {
    int n = 0;
    for (int c = 0; c < e->C; c++) n += e->core_owner[c] == agent_id;
    return n;
}

/* JobCollection.insertJob (world.py:123-133) */
static void insert_job(mso_env* e, int agent, mso_job job) {
    if (e->free_slots[agent] > 0) {
        for (int s = 0; s < e->L; s++) {
            if (e->coll[agent * e->L + s].empty) {
                e->coll[agent * e->L + s] = job;
                e->free_slots[agent] -= 1;
                break;
            }
        }
    } else {
        e->flags |= MS_FLAG_COLLECTION_FULL; /* the reference raises here */
    }
}

/* JobCollection.removeAndReturnEntry (world.py:135-141) */
static mso_job remove_entry(mso_env* e, int agent, int slot) {
    mso_job r = e->coll[agent * e->L + slot];
    e->coll[agent * e->L + slot] = empty_job();
    e->free_slots[agent] += 1;
    return r;
}

/* World.executeAnOffer (world.py:261-293) with Core.dispatchNewJobAndReturnOldOne (:61-76) */
static void execute_offer(mso_env* e, int offer_id, ms_accept_rec* acc_rec, int* n_exec,
                          double* quality, int* n_quality) {
    mso_offer* off = NULL;
    for (int i = 0; i < e->n_offers; i++)
        if (e->offers[i].offer_id == offer_id) off = &e->offers[i];
    if (!off) return;
    int c = off->core_id - 1;
    if (off->recipient != e->core_owner[c]) { /* ownership guard world.py:266 */
        e->flags |= MS_FLAG_GUARD;
        return;
    }
    int offerer = off->offerer - 1;
    mso_job new_job = remove_entry(e, offerer, off->queue_pos);
    new_job.wait = 0; /* world.py:276 */
    mso_job old_job = e->core_job[c].empty ? empty_job() : e->core_job[c];
    e->core_job[c] = new_job;
    e->core_owner[c] = new_job.empty ? 0 : off->offerer; /* newJob.ownerID == offerer (jobs stay with their creator's collection) */
    if (off->recipient != 0) insert_job(e, off->recipient - 1, old_job); /* world.py:278-281 */
    /* liability entry (deepcopy with round = world.round), appendleft (world.py:285-289) */
    if (e->liab_n[c] < e->cap) {
        mso_offer le = *off;
        le.round = e->round;
        e->liab[c * e->cap + e->liab_n[c]] = le;
        e->liab_n[c] += 1;
    } else {
        e->flags |= MS_FLAG_LIABILITY_OVERFLOW;
    }
    /* world.acceptedOffers.append (world.py:293) */
    ms_accept_rec* r = &acc_rec[c];
    r->valid = 1;
    r->offerer = (int8_t)off->offerer;
    r->recipient = (int8_t)off->recipient;
    r->slot = (int8_t)off->queue_pos;
    r->price = (int8_t)off->price;
    r->nec_time = (int8_t)off->nec_time;
    r->prio = (int8_t)off->prio1;
    r->kind = (int8_t)off->kind;
    r->order = (int8_t)(*n_exec);
    r->round = e->round;
    *n_exec += 1;
    /* calculateAverageAcceptionQuality (SchedulingEnvironment.py:174-192), non-auctioneer offers */
    if (off->recipient != 0) {
        double q = ((double)off->price / (double)off->nec_time) -
                   ((e->former_prio[c] != -1) ? ((double)e->former_prio[c] / (double)e->former_len[c]) : 0.0);
        q *= 10;
        quality[(*n_quality)++] = q;
    }
}

/* calculateRewardRatio (HardcodedModules.py:5-13), as an exact fraction num/den */
static void reward_ratio(int p, int n, long* num, long* den) {
    if (p == -1 || n == -1 || p == -2 || n == -2) {
        *num = -1;
        *den = 1;
    } else {
        *num = p;
        *den = n;
        if (*den < 0) {
            *num = -*num;
            *den = -*den;
        }
    }
}

/* a/b > c/d for b,d > 0 (exact; equals the double comparison for these ranges) */
static int frac_gt(long a, long b, long c, long d) { return a * d > c * b; }
static int frac_eq(long a, long b, long c, long d) { return a * d == c * b; }

/* HardcodedAuctioneerAcceptor.selectAction (HardcodedModules.py:54-78) on the
 * auctioneer observation of each core (Auctioneer.py:34-77), cores in order
 * (Auctioneer.getAuctioneerAction Auctioneer.py:95-102). */
void mso_auctioneer_actions(mso_env* e, int32_t* out) {
    long num[MS_MAX_OFFERS + 1], den[MS_MAX_OFFERS + 1];
    for (int c = 0; c < e->C; c++) {
        if (e->core_owner[c] != 0) { /* ownership flag == 0 */
            out[c] = e->O;
            continue;
        }
        /* own ratio: the auctioneer's core holds the empty job -> (-1,-1) -> -1 */
        long own_n, own_d;
        reward_ratio(e->core_job[c].prio, e->core_job[c].rem, &own_n, &own_d);
        int k = 0;
        for (int i = 0; i < e->n_offers; i++) {
            const mso_offer* o = &e->offers[i];
            if (o->recipient == 0 && o->core_id == c + 1) {
                reward_ratio(o->price, o->nec_time, &num[k], &den[k]);
                k++;
            }
        }
        for (; k < e->O; k++) { /* (-2,-2) padding */
            num[k] = -1;
            den[k] = 1;
        }
        long mn = num[0], md = den[0];
        for (int i = 1; i < e->O; i++)
            if (frac_gt(num[i], den[i], mn, md)) {
                mn = num[i];
                md = den[i];
            }
        if (frac_gt(mn, md, own_n, own_d)) {
            int cands[MS_MAX_OFFERS];
            int nc = 0;
            for (int i = 0; i < e->O; i++)
                if (frac_eq(num[i], den[i], mn, md)) cands[nc++] = i;
            /* random.sample(cands, 1) -> one _randbelow(len) (random.py:480-494) */
            out[c] = cands[mt_randbelow(&e->rng, (uint32_t)nc)];
        } else {
            out[c] = e->O;
        }
    }
}

/* World.processOneTimestepAndUpdateOwnership (world.py:336-367) */
typedef struct {
    int valid, owner, reward, ts;
} mso_term;

static void tick(mso_env* e, mso_term* term, ms_term_rec* trec) {
    for (int c = 0; c < e->C; c++) {
        term[c].valid = 0;
        if (trec) memset(&trec[c], 0, sizeof(ms_term_rec));
        mso_job* j = &e->core_job[c];
        if (!j->empty) {
            j->rem -= 1;
            if (j->rem == 0) {
                term[c].valid = 1;
                term[c].owner = e->core_owner[c];
                term[c].reward = e->cfg.reward_multiplier * j->prio;
                term[c].ts = e->round + 1;
                if (trec) {
                    trec[c].valid = 1;
                    trec[c].owner = (int8_t)e->core_owner[c];
                    trec[c].prio = (int8_t)j->prio;
                    trec[c].init_len = (int8_t)j->init_len;
                    trec[c].dwell = e->round - j->birth;
                }
                *j = empty_job(); /* Core.assignCoreToAuctioneer world.py:57-59 */
                e->core_owner[c] = 0;
            }
        }
    }
}

/* createFixPriceOfferObjectsFromActions (world.py:406-443) /
 * createFreePriceOfferObjectsFromActions (world.py:445-478) */
static void create_offers(mso_env* e, const int32_t* off_core, const int32_t* off_price) {
    e->n_offers = 0;
    int next_id = 1; /* Offer.offerID = 1 (world.py:325) */
    for (int a = 0; a < e->N; a++) {
        for (int s = 0; s < e->L; s++) {
            int action = off_core[a * e->L + s];
            int core_id = action + 1;
            int cidx = (core_id >= 1 && core_id <= e->C) ? core_id - 1 : -1;
            mso_job* job = &e->coll[a * e->L + s];
            int price;
            if (e->cfg.free_prices) {
                price = off_price[a * e->L + s];
            } else {
                /* listOfFixPrices[jobKind]; an empty job's kind -1 indexes the last price */
                int k = job->kind >= 0 ? job->kind : e->cfg.n_fix_prices - 1;
                price = e->cfg.fix_price[k];
            }
            if (cidx >= 0 && !job->empty && !job->wait) {
                mso_offer* o = &e->offers[e->n_offers++];
                o->offer_id = next_id++;
                o->offerer = a + 1;
                o->recipient = e->core_owner[cidx];
                o->core_id = cidx + 1;
                o->queue_pos = s;
                o->price = price;
                o->nec_time = job->rem;
                o->prio1 = job->prio;
                o->kind = job->kind;
                o->round = e->round;
                job->wait = 1;
            } else {
                job->wait = 0;
            }
        }
    }
}

/* World.fillQueuesWithNewRandomJobs (world.py:369-376) + Agent.fillCollectionRandomly (Agent.py:50-70) */
static void spawn(mso_env* e) {
    int k = e->cfg.new_jobs_per_round;
    for (int a = 0; a < e->N; a++) {
        if (owned_cores(e, a + 1) + k <= e->free_slots[a]) {
            for (int t = 0; t < k; t++) {
                double u = mt_random(&e->rng);
                int kind = -1;
                for (int i = 0; i < e->cfg.n_kinds; i++)
                    if (u < e->cfg.acc_probability[i]) {
                        kind = i;
                        break;
                    }
                if (kind < 0) { /* reference: UnboundLocalError / stale index */
                    kind = e->cfg.n_kinds - 1;
                    e->flags |= MS_FLAG_SPAWN_EDGE;
                }
                mso_job j;
                j.empty = 0;
                j.kind = kind;
                j.prio = e->cfg.job_priority[kind];
                j.rem = e->cfg.job_length[kind];
                j.init_len = e->cfg.job_length[kind];
                j.birth = e->round;
                j.wait = 0;
                insert_job(e, a, j);
            }
        }
    }
}

/* Python round(): float64 product then round-half-even (Reward.py:200-201) */
static long traded_reward(int price, int nec, int t) {
    double ratio = (double)price / (double)nec;
    double x = ratio * (double)t;
    return (long)nearbyint(x);
}

/* getDividedFixedPricesReward (Reward.py:146-212) / getDividedFreePricesReward (Reward.py:6-89) */
static void rewards(mso_env* e, const mso_term* term, const ms_accept_rec* acc_rec, mso_step_out* out) {
    int N = e->N, C = e->C, L = e->L;
    for (int i = 0; i < N * L; i++) {
        if (out->offer) out->offer[i] = 0;
        if (out->price) out->price[i] = 0;
    }
    for (int i = 0; i < N * C; i++) out->acceptor[i] = 0;
    for (int c = 0; c < C; c++) out->auctioneer[c] = 0;
    for (int a = 0; a < N; a++) out->agent[a] = 0;
    out->termination_revenue = 0;
    /* offer-side rewards from world.acceptedOffers */
    for (int c = 0; c < C; c++) {
        const ms_accept_rec* r = &acc_rec[c];
        if (!r->valid) continue;
        int idx = (r->offerer - 1) * L + r->slot;
        if (!e->cfg.free_prices) {
            if (out->offer) out->offer[idx] = r->prio; /* Reward.py:164-170 */
        } else {
            double pc;
            int diff = r->prio - r->price;
            if (e->cfg.commercial_reward)
                pc = diff == 0 ? e->cfg.net_zero_offer_reward : (double)diff; /* Reward.py:29-33 */
            else
                pc = diff >= 0 ? (double)r->prio : (double)diff; /* Reward.py:43-47 */
            if (out->offer) out->offer[idx] = r->prio;
            if (out->price) out->price[idx] = pc;
        }
    }
    /* liability chains of terminated cores, cores in order (jobTerminationInfo order) */
    for (int c = 0; c < C; c++) {
        if (!term[c].valid) continue;
        int owner = term[c].owner;
        out->acceptor[(owner - 1) * C + c] = term[c].reward;
        if (!e->cfg.free_prices) {
            out->agent[owner - 1] += term[c].reward;
            out->termination_revenue += term[c].reward;
        }
        int last_ts = term[c].ts, tm = 0;
        for (int k = e->liab_n[c] - 1; k >= 0; k--) { /* newest first */
            const mso_offer* le = &e->liab[c * e->cap + k];
            tm += last_ts - le->round;
            last_ts = le->round;
            long traded = traded_reward(le->price, le->nec_time, tm);
            out->acceptor[(le->offerer - 1) * C + c] -= traded;
            out->agent[le->offerer - 1] -= traded;
            if (le->recipient > 0) {
                out->agent[le->recipient - 1] += traded;
                out->acceptor[(le->recipient - 1) * C + c] += traded;
            }
            if (le->recipient == 0) out->auctioneer[c] = traded;
        }
        e->liab_n[c] = 0; /* resetLiabilityListForACore */
    }
}

int mso_step(mso_env* e, const int32_t* acc_act, const int32_t* off_core, const int32_t* off_price,
             const int32_t* auct_act, mso_step_out* out) {
    int N = e->N, C = e->C, O = e->O;
    int32_t auct[MS_MAX_CORES];
    /* the driver asks the auctioneer before env.step (trainPPO.py:162) */
    if (auct_act) {
        for (int c = 0; c < C; c++) auct[c] = auct_act[c];
    } else {
        mso_auctioneer_actions(e, auct);
    }
    ms_accept_rec acc_rec[MS_MAX_CORES];
    memset(acc_rec, 0, sizeof(acc_rec));
    int n_exec = 0;
    double quality[MS_MAX_CORES];
    int n_quality = 0;
    /* step1 (world.py:295-334); the liability resets of :309-310 are no-ops here
     * because getRewards already reset those chains at the end of the last step */
    /* executeAgentAcceptions1 (world.py:391-404): ids = correspondingOfferIDs of the last obs */
    for (int a = 0; a < N; a++) {
        for (int c = 0; c < C; c++) {
            int idx = acc_act[a * C + c];
            if (idx >= 0 && idx < O) {
                int k = 0, id = -2;
                for (int i = 0; i < e->n_offers; i++) {
                    if (e->offers[i].recipient == a + 1 && e->offers[i].core_id == c + 1) {
                        if (k == idx) {
                            id = e->offers[i].offer_id;
                            break;
                        }
                        k++;
                    }
                }
                if (id > 0) execute_offer(e, id, acc_rec, &n_exec, quality, &n_quality);
            } else if (idx != O) {
                e->flags |= MS_FLAG_BAD_ACTION;
            }
        }
    }
    /* executeAuctioneerAcceptions (world.py:378-389) */
    for (int c = 0; c < C; c++) {
        int idx = auct[c];
        if (idx >= 0 && idx < O) {
            int k = 0, id = -2;
            for (int i = 0; i < e->n_offers; i++) {
                if (e->offers[i].recipient == 0 && e->offers[i].core_id == c + 1) {
                    if (k == idx) {
                        id = e->offers[i].offer_id;
                        break;
                    }
                    k++;
                }
            }
            if (id > 0) execute_offer(e, id, acc_rec, &n_exec, quality, &n_quality);
        } else if (idx != O) {
            e->flags |= MS_FLAG_BAD_ACTION;
        }
    }
    mso_term term[MS_MAX_CORES];
    tick(e, term, out ? out->terminated : NULL);
    create_offers(e, off_core, off_price);
    spawn(e);
    e->round += 1;
    /* getRewards after the observations (SchedulingEnvironment.py:60-62) */
    if (out) {
        if (out->accepted) memcpy(out->accepted, acc_rec, sizeof(ms_accept_rec) * C);
        for (int i = 0; i < n_quality; i++) out->quality[i] = quality[i];
        out->n_quality = n_quality;
        rewards(e, term, acc_rec, out);
    } else {
        mso_step_out tmp;
        double* off = (double*)calloc((size_t)N * e->L, sizeof(double));
        double* pr = (double*)calloc((size_t)N * e->L, sizeof(double));
        int64_t* ar = (int64_t*)calloc((size_t)N * C, sizeof(int64_t));
        int64_t au[MS_MAX_CORES], ag[MS_MAX_AGENTS];
        tmp.offer = off;
        tmp.price = pr;
        tmp.acceptor = ar;
        tmp.auctioneer = au;
        tmp.agent = ag;
        rewards(e, term, acc_rec, &tmp);
        free(off);
        free(pr);
        free(ar);
    }
    /* formerCorePrios/Lengths (SchedulingEnvironment.py:70-71) */
    for (int c = 0; c < C; c++) {
        e->former_prio[c] = e->core_job[c].prio;
        e->former_len[c] = e->core_job[c].rem;
    }
    return 0;
}

/* DividedAgent.gatherObservations (Agent.py:148-300) + gatherDividedAuctioneerObservation
 * (Auctioneer.py:20-77) */
static void acceptor_row(const mso_env* e, int recipient, int c, int32_t* obs, int32_t* ids) {
    int own = e->core_owner[c] == recipient;
    int w = 0;
    obs[w++] = own;
    obs[w++] = own ? e->core_job[c].prio : -1;
    obs[w++] = own ? e->core_job[c].rem : -1;
    int k = 0;
    for (int i = 0; i < e->n_offers; i++) {
        const mso_offer* o = &e->offers[i];
        if (o->recipient == recipient && o->core_id == c + 1) {
            obs[w++] = o->price;
            obs[w++] = o->nec_time;
            if (ids) ids[k] = o->offer_id;
            k++;
        }
    }
    for (; k < e->O; k++) {
        obs[w++] = -2;
        obs[w++] = -2;
        if (ids) ids[k] = -2;
    }
}

void mso_observe(const mso_env* e, int32_t* acc_obs, int32_t* acc_ids, int32_t* off_obs,
                 int32_t* auct_obs, int32_t* auct_ids) {
    int N = e->N, C = e->C, L = e->L, O = e->O;
    int D_acc = 3 + 2 * O, D_off = 2 * C + 2;
    for (int a = 0; a < N; a++) {
        for (int c = 0; c < C; c++) {
            int32_t tmp_obs[3 + 2 * MS_MAX_OFFERS];
            int32_t tmp_ids[MS_MAX_OFFERS];
            acceptor_row(e, a + 1, c, tmp_obs, tmp_ids);
            if (acc_obs) memcpy(acc_obs + ((size_t)a * C + c) * D_acc, tmp_obs, sizeof(int32_t) * D_acc);
            if (acc_ids) memcpy(acc_ids + ((size_t)a * C + c) * O, tmp_ids, sizeof(int32_t) * O);
        }
        for (int s = 0; s < L; s++) {
            if (!off_obs) break;
            int32_t* row = off_obs + ((size_t)a * L + s) * D_off;
            for (int c = 0; c < C; c++) {
                row[2 * c] = e->core_job[c].prio;
                row[2 * c + 1] = e->core_job[c].rem;
            }
            row[2 * C] = e->coll[a * L + s].prio;
            row[2 * C + 1] = e->coll[a * L + s].rem;
        }
    }
    for (int c = 0; c < C; c++) {
        int32_t tmp_obs[3 + 2 * MS_MAX_OFFERS];
        int32_t tmp_ids[MS_MAX_OFFERS];
        acceptor_row(e, 0, c, tmp_obs, tmp_ids);
        if (auct_obs) memcpy(auct_obs + (size_t)c * D_acc, tmp_obs, sizeof(int32_t) * D_acc);
        if (auct_ids) memcpy(auct_ids + (size_t)c * O, tmp_ids, sizeof(int32_t) * O);
    }
}

/* ------------------------------------------------------------------------- */
/* canonical state export / import */

void mso_export(const mso_env* e, const ms_state_host* o) {
    int N = e->N, C = e->C, L = e->L;
    if (o->round) o->round[0] = e->round;
    if (o->flags) o->flags[0] = e->flags;
    for (int c = 0; c < C; c++) {
        if (o->core_owner) o->core_owner[c] = e->core_owner[c];
        if (o->core_kind) o->core_kind[c] = e->core_job[c].kind;
        if (o->core_rem) o->core_rem[c] = e->core_job[c].rem;
        if (o->core_birth) o->core_birth[c] = e->core_job[c].empty ? -1 : e->core_job[c].birth;
        if (o->liab_n) o->liab_n[c] = e->liab_n[c];
        if (o->liab) {
            for (int k = 0; k < e->cap; k++) {
                int32_t* d = o->liab + ((size_t)c * e->cap + k) * 5;
                if (k < e->liab_n[c]) {
                    const mso_offer* le = &e->liab[c * e->cap + k];
                    d[0] = le->offerer;
                    d[1] = le->recipient;
                    d[2] = le->price;
                    d[3] = le->nec_time;
                    d[4] = le->round;
                } else {
                    d[0] = d[1] = d[2] = d[3] = d[4] = 0;
                }
            }
        }
    }
    for (int i = 0; i < N * L; i++) {
        const mso_job* j = &e->coll[i];
        if (o->slot_kind) o->slot_kind[i] = j->kind;
        if (o->slot_rem) o->slot_rem[i] = j->rem;
        if (o->slot_wait) o->slot_wait[i] = j->wait;
        if (o->slot_birth) o->slot_birth[i] = j->empty ? -1 : j->birth;
        if (o->offer_core) o->offer_core[i] = -1;
        if (o->offer_recip) o->offer_recip[i] = 0;
        if (o->offer_price) o->offer_price[i] = 0;
    }
    for (int i = 0; i < e->n_offers; i++) {
        const mso_offer* of = &e->offers[i];
        int idx = (of->offerer - 1) * L + of->queue_pos;
        if (o->offer_core) o->offer_core[idx] = of->core_id - 1;
        if (o->offer_recip) o->offer_recip[idx] = of->recipient;
        if (o->offer_price) o->offer_price[idx] = of->price;
    }
    if (o->mt) memcpy(o->mt, e->rng.mt, sizeof(e->rng.mt));
    if (o->mt_index) o->mt_index[0] = e->rng.mti;
}

int mso_import(mso_env* e, const ms_state_host* in) {
    int N = e->N, C = e->C, L = e->L;
    e->round = in->round[0];
    e->flags = in->flags ? in->flags[0] : 0;
    for (int c = 0; c < C; c++) {
        int k = in->core_kind[c];
        if (k < 0) {
            e->core_job[c] = empty_job();
            e->core_owner[c] = 0;
        } else {
            mso_job j;
            j.empty = 0;
            j.kind = k;
            j.prio = e->cfg.job_priority[k];
            j.rem = in->core_rem[c];
            j.init_len = e->cfg.job_length[k];
            j.birth = in->core_birth[c];
            j.wait = 0;
            e->core_job[c] = j;
            e->core_owner[c] = in->core_owner[c];
        }
        e->former_prio[c] = e->core_job[c].prio;
        e->former_len[c] = e->core_job[c].rem;
        e->liab_n[c] = in->liab_n[c];
        for (int q = 0; q < in->liab_n[c] && q < e->cap; q++) {
            const int32_t* d = in->liab + ((size_t)c * e->cap + q) * 5;
            mso_offer* le = &e->liab[c * e->cap + q];
            memset(le, 0, sizeof(*le));
            le->offerer = d[0];
            le->recipient = d[1];
            le->price = d[2];
            le->nec_time = d[3];
            le->round = d[4];
            le->core_id = c + 1;
        }
    }
    for (int a = 0; a < N; a++) e->free_slots[a] = 0;
    for (int i = 0; i < N * L; i++) {
        int k = in->slot_kind[i];
        if (k < 0) {
            e->coll[i] = empty_job();
            e->free_slots[i / L] += 1;
        } else {
            mso_job j;
            j.empty = 0;
            j.kind = k;
            j.prio = e->cfg.job_priority[k];
            j.rem = in->slot_rem[i];
            j.init_len = e->cfg.job_length[k];
            j.birth = in->slot_birth[i];
            j.wait = in->slot_wait[i];
            e->coll[i] = j;
        }
    }
    e->n_offers = 0;
    for (int i = 0; i < N * L; i++) {
        if (in->offer_core[i] < 0) continue;
        mso_offer* o = &e->offers[e->n_offers];
        o->offer_id = e->n_offers + 1;
        o->offerer = i / L + 1;
        o->recipient = in->offer_recip[i];
        o->core_id = in->offer_core[i] + 1;
        o->queue_pos = i % L;
        o->price = in->offer_price[i];
        o->nec_time = e->coll[i].rem;
        o->prio1 = e->coll[i].prio;
        o->kind = e->coll[i].kind;
        o->round = e->round - 1;
        e->n_offers++;
    }
    memcpy(e->rng.mt, in->mt, sizeof(e->rng.mt));
    e->rng.mti = in->mt_index[0];
    return 0;
}

int64_t mso_round(const mso_env* e) { return e->round; }
uint32_t mso_flags(const mso_env* e) { return e->flags; }
uint32_t mso_genrand(mso_env* e) { return mt_genrand(&e->rng); }
double mso_random(mso_env* e) { return mt_random(&e->rng); }
uint32_t mso_randbelow(mso_env* e, uint32_t n) { return mt_randbelow(&e->rng, n); }

/* ------------------------------------------------------------------------- */
/* batched CPU baseline: same I/O shapes as the device ABI */

int mso_step_batch(mso_env** envs, int64_t E, const int8_t* acc_act, const int8_t* off_core,
                   const int8_t* off_price, int8_t* acc_obs, int8_t* off_obs, int32_t acc_stride,
                   int32_t off_stride, float* offer_rew, float* price_rew, int32_t* acc_rew, int threads) {
    (void)threads;
    int64_t e;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1) if (threads != 1)
    for (e = 0; e < E; e++) {
        mso_env* env = envs[e];
        int N = env->N, C = env->C, L = env->L, O = env->O;
        int D_acc = 3 + 2 * O, D_off = 2 * C + 2;
        int32_t aa[MS_MAX_AGENTS * MS_MAX_CORES], oc[MS_MAX_AGENTS * MS_MAX_COLLECTION],
            op[MS_MAX_AGENTS * MS_MAX_COLLECTION];
        for (int i = 0; i < N * C; i++) aa[i] = acc_act[e * N * C + i];
        for (int i = 0; i < N * L; i++) {
            oc[i] = off_core[e * N * L + i];
            op[i] = off_price ? off_price[e * N * L + i] : 0;
        }
        double* orw = (double*)malloc(sizeof(double) * N * L * 2);
        int64_t* arw = (int64_t*)malloc(sizeof(int64_t) * N * C);
        int64_t au[MS_MAX_CORES], ag[MS_MAX_AGENTS];
        ms_accept_rec accr[MS_MAX_CORES];
        ms_term_rec termr[MS_MAX_CORES];
        double q[MS_MAX_CORES];
        mso_step_out out;
        memset(&out, 0, sizeof(out));
        out.offer = orw;
        out.price = orw + N * L;
        out.acceptor = arw;
        out.auctioneer = au;
        out.agent = ag;
        out.accepted = accr;
        out.terminated = termr;
        out.quality = q;
        mso_step(env, aa, oc, off_price ? op : NULL, NULL, &out);
        int32_t* ao = (int32_t*)malloc(sizeof(int32_t) * (N * C * D_acc + N * L * D_off));
        int32_t* oo = ao + N * C * D_acc;
        mso_observe(env, ao, NULL, oo, NULL, NULL);
        if (acc_obs)
            for (int r = 0; r < N * C; r++)
                for (int d = 0; d < acc_stride; d++)
                    acc_obs[(e * N * C + r) * (int64_t)acc_stride + d] = d < D_acc ? (int8_t)ao[r * D_acc + d] : 0;
        if (off_obs)
            for (int r = 0; r < N * L; r++)
                for (int d = 0; d < off_stride; d++)
                    off_obs[(e * N * L + r) * (int64_t)off_stride + d] = d < D_off ? (int8_t)oo[r * D_off + d] : 0;
        for (int i = 0; i < N * L; i++) {
            if (offer_rew) offer_rew[e * N * L + i] = (float)orw[i];
            if (price_rew) price_rew[e * N * L + i] = (float)orw[N * L + i];
        }
        for (int i = 0; i < N * C; i++)
            if (acc_rew) acc_rew[e * N * C + i] = (int32_t)arw[i];
        free(ao);
        free(orw);
        free(arw);
    }
    return 0;
}
