// ms_layout.h — per-env state record layout and launch parameters shared by
// the host ABI (capi.cpp) and the HIP kernels.
//
// One env replica's state lives in one contiguous record in HBM (the
// [env][field][agent/core/slot] layout: env-major so that the one wave that
// steps an env reads and writes it with a few coalesced dword accesses):
//
//   int32  round, flags, mti, pad                       16 B
//   int8   core_owner[C], core_kind[C], core_rem[C], liab_n[C]   (each padded to 4)
//   int32  core_birth[C]
//   int8   slot_kind[NL], slot_rem[NL], slot_wait[NL],
//          offer_core[NL], offer_recip[NL], offer_price[NL]        (each padded to 4)
//   int32  slot_birth[NL]
//
// Beside it: liability chains [E][C][cap] of 8-byte entries and the MT19937
// state words [E][624].
#pragma once

#include <stdint.h>

#include "../../include/marlsched.h"

namespace ms {

constexpr int kWave = 64;
constexpr int kMtN = 624;
constexpr int kMtM = 397;

struct Liab {  // one liabilityList entry (world.py:285-289)
    int8_t offerer, recipient, price, nec;
    int32_t round;
};

inline constexpr int32_t align4(int32_t x) { return (x + 3) & ~3; }
inline constexpr int32_t align16(int32_t x) { return (x + 15) & ~15; }
// w / d == umulhi(w, magic_div(d)) for every w < 2^32 / d and d >= 2 (d == 1 is the emitters'
// special case: the quotient is w).
inline constexpr uint32_t magic_div(uint32_t d) { return d < 2 ? 0u : (uint32_t)(0x100000000ull / d + 1); }

// The shape-derived part of the launch parameters: sizes, the record layout and the LDS plan. It
// depends only on (N, C, L, newJobsPerRound), so the env kernels can take it either from the
// kernel arguments or, for the BASELINE shapes, as a compile-time constant (make_geom in a
// constexpr context): every offset then folds into the instructions' immediates and every loop
// over agents / cores / slots has a constant trip count.
struct Geom {
    // shapes
    int32_t N, C, L, NL, O;
    int32_t d_acc, acc_stride, d_off, off_stride;
    // record byte offsets
    int32_t o_core_owner, o_core_kind, o_core_rem, o_liab_n, o_core_birth;
    int32_t o_slot_kind, o_slot_rem, o_slot_wait, o_offer_core, o_offer_recip, o_offer_price,
        o_slot_birth;
    int32_t rec_bytes;
    // LDS carve-up (byte offsets into dynamic shared memory), sized to the config so that
    // small envs keep many waves per CU in flight
    int32_t s_rec, s_act_acc, s_act_off, s_act_price, s_act_auct, s_accr, s_offr, s_pricer,
        s_spawn_kind, s_scratch, s_total;
    int32_t s_mc, s_mr, s_newle, s_exec, s_key, s_auct, s_agentr, s_credit, s_auctr, s_rank, s_fresh, s_misc;
    // observation scratch (offsets inside s_scratch): C owner rows + the foreign row
    // [C+1][acc_stride], the source-row dword offset of every acceptor row [N*C] u16, the
    // offer-row template [off_stride] and the slot pairs [NL] u16
    int32_t scratch_bytes, s_rowsel, s_otmpl, s_slotpair;
    // w / nw == umulhi(w, mag) for the dword counts of one env's acceptor / offer rows
    uint32_t mag_acc, mag_off;
};

inline constexpr Geom make_geom(int32_t n_agents, int32_t n_cores, int32_t coll_len, int32_t new_jobs) {
    Geom p{};
    p.N = n_agents;
    p.C = n_cores;
    p.L = coll_len;
    p.NL = p.N * p.L;
    p.O = p.NL;
    p.d_acc = 3 + 2 * p.O;
    p.acc_stride = align4(p.d_acc);
    p.d_off = 2 * p.C + 2;
    p.off_stride = align4(p.d_off);
    int32_t o = 16;
    p.o_core_owner = o; o += align4(p.C);
    p.o_core_kind = o; o += align4(p.C);
    p.o_core_rem = o; o += align4(p.C);
    p.o_liab_n = o; o += align4(p.C);
    p.o_core_birth = o; o += 4 * p.C;
    p.o_slot_kind = o; o += align4(p.NL);
    p.o_slot_rem = o; o += align4(p.NL);
    p.o_slot_wait = o; o += align4(p.NL);
    p.o_offer_core = o; o += align4(p.NL);
    p.o_offer_recip = o; o += align4(p.NL);
    p.o_offer_price = o; o += align4(p.NL);
    p.o_slot_birth = o; o += 4 * p.NL;
    p.rec_bytes = align16(o);
    // LDS plan
    int32_t s = 0;
    p.s_rec = s; s += p.rec_bytes;
    p.s_act_acc = s; s += align4(p.N * p.C);
    p.s_act_off = s; s += align4(p.NL);
    p.s_act_price = s; s += align4(p.NL);
    p.s_act_auct = s; s += align4(p.C);
    p.s_accr = s; s += 4 * p.N * p.C;          // acceptorNetRewards int32
    p.s_offr = s; s += 4 * p.NL;               // offer / coreChooser rewards f32
    p.s_pricer = s; s += 4 * p.NL;             // priceChooser rewards f32
    p.s_spawn_kind = s; s += align4(p.N * (new_jobs > 0 ? new_jobs : 1));
    s = align16(s);
    p.s_mc = s; s += 16 * p.C;                 // offer masks per core (M128)
    p.s_mr = s; s += 16 * (p.N + 1);           // offer masks per recipient
    p.s_newle = s; s += 8 * p.C;               // this round's liability entry per core
    p.s_agentr = s; s += 4 * p.N;              // agentReward
    p.s_credit = s; s += 4 * p.N;              // chain credits received (aggregated acceptor rewards)
    p.s_auctr = s; s += 4 * p.C;               // auctioneerReward
    p.s_exec = s; s += align4(2 * p.C);        // executed slot per core
    p.s_key = s; s += align4(2 * p.C);         // execution order key
    p.s_auct = s; s += align4(2 * p.C);        // auctioneer action per core
    p.s_rank = s; s += align4(p.C);            // cores in execution order
    p.s_fresh = s; s += align4(p.C);           // s_newle[c] is the chain's newest entry
    p.s_misc = s; s += 16;                     // flags, n_exec
    s = align16(s);
    p.s_scratch = s;
    p.s_rowsel = (p.C + 1) * p.acc_stride;
    p.s_otmpl = align4(p.s_rowsel + 2 * p.N * p.C);
    p.s_slotpair = p.s_otmpl + p.off_stride;
    p.scratch_bytes = align16(p.s_slotpair + 2 * p.NL);
    s += p.scratch_bytes;
    p.s_total = s;
    p.mag_acc = magic_div(p.acc_stride / 4);
    p.mag_off = magic_div(p.off_stride / 4);
    return p;
}

struct Params : Geom {
    int32_t K, cap;
    // config (world.py:211-246, Reward.py)
    int32_t prio[MS_MAX_KINDS];
    int32_t len[MS_MAX_KINDS];
    double acc[MS_MAX_KINDS];
    int32_t fix[MS_MAX_KINDS];
    int32_t n_fix;
    int32_t free_prices, commercial, new_jobs, mult;
    int32_t ep_len;  // episodeLength (world.py:243): the metrics slot of a round
    float net_zero;
};

// device pointers of one ms_env_step call
struct StepIO {
    const int8_t* act_acc;
    const int8_t* act_off;
    const int8_t* act_price;
    const int8_t* act_auct;
    int8_t* obs_acc;
    int8_t* obs_off;
    int8_t* obs_auct;
    int8_t* obs_crow;  // [E][C][acc_stride] owner row of every core, or NULL
    int8_t* obs_cown;  // [E][C] core owners, or NULL
    float* rew_offer;
    float* rew_price;
    int32_t* rew_acc;
    int32_t* rew_auct;
    int32_t* rew_agent;
    int32_t* rew_agg_off;
    int32_t* rew_agg_acc;
    ms_accept_rec* ev_acc;
    ms_term_rec* ev_term;
    uint32_t* err_word;  // host-coherent sticky word: set to 1 by a round raising a fatal flag
    unsigned long long* span;  // [waves][2] or NULL: each wave's start / end (s_memrealtime)
    ms_env_metrics* metrics;   // [slots][E] episode accumulators or NULL
    int32_t metrics_slots;
};

// the fused next-round acting of ms_env_step_act (env_kernels.hip fused_act)
struct FusedAct {
    ms_mlp_params off, acc;
    const int8_t* common;
    uint64_t seed, off_offset, acc_offset;
    const uint64_t* offset_dev;
    int8_t* off_action;
    float* off_logprob;
    int8_t* acc_action;
    float* acc_logprob;
};

// per-round byte strides of k_env_rollout_act (ms_round_strides)
struct RoundStride {
    int64_t act_acc, act_off, obs_crow, obs_cown, obs_off, rew_offer, rew_acc, rew_agent, rew_auct;
    int64_t off_action, off_logprob, acc_action, acc_logprob;
    uint64_t offset_step;
};

// the fused next-round acting of a locally shared free-price rollout (ms_env_rollout_act_free,
// env_kernels.hip act_free): one core chooser, price chooser and acceptor net per agent
struct FusedActFree {
    ms_mlp_params core, price, acc;
    const int8_t* common;
    const float* ptab;       // price table [N][pkeys][PriceTW] (ms_price_table)
    const int16_t* pdigit;   // [4][256] key digit of byte value v at position p, -1: not tabulated
    int32_t pkeys;
    uint64_t seed, off_offset, acc_offset;
    const uint64_t* offset_dev;
    int8_t* core_action;     // [E][N*L]
    float* core_logprob;
    int8_t* price_state;     // [E][N*L][4]
    int8_t* price_action;
    float* price_logprob;
    int8_t* env_price;       // [E][N*L]: the next round's offer_price actions (one buffer, every round)
    int8_t* acc_action;      // [E][N*C]
    float* acc_logprob;
    int8_t* own_action;      // [E][C] the owned items by core (NULL: in acc_action / acc_logprob directly)
    float* own_logprob;
};

// per-round byte strides of k_env_rollout_act_free (ms_round_strides_free)
struct RoundStrideFree {
    int64_t act_acc, act_off, obs_crow, obs_cown, obs_off, rew_offer, rew_price, rew_acc, rew_agent, rew_auct;
    int64_t core_action, core_logprob, price_state, price_action, price_logprob, acc_action, acc_logprob;
    uint64_t offset_step;
    int64_t own_action, own_logprob;
};

// The workgroup LDS of k_env_rollout_act_free: the env slices of its kFreeEPW * N replicas (wave w steps
// replicas kFreeEPW * w ..), then the act area: the price table's key digits (one copy per workgroup) and per
// wave (= agent) its list of owned-core acceptor rows.
constexpr int kFreeEPW = 4;        // replicas per wave (16 lanes each)
constexpr int kFreeListCap = 96;   // < 32 carried + one 64-item step
constexpr int kFreeTabDw = 68;     // [32 running sums][32 log-probs][S][last nonzero][2 pad] (Head<2>::table)
struct FreeLds {
    int32_t pdig, list, accx, pace, total;
};
inline constexpr FreeLds free_lds(const Geom& g) {
    FreeLds f{};
    f.pdig = align16(kFreeEPW * g.N * g.s_total);
    f.list = f.pdig + 4 * 256 * 2;
    f.accx = align16(f.list + g.N * kFreeListCap * 6);  // int16 item + f32 uniform per entry
    // (by-core mode) the replicas' acceptor actions [kFreeEPW * N][N * C]: the acting writes its owned items, the
    // next env round stages its owners' from here (outside the wave slots the MT refill may overwrite)
    f.pace = f.accx + align4(kFreeEPW * g.N * g.N * g.C);
    f.total = f.pace + 4 * 8;  // (MS_FREE_PRIO bit 2) each wave's count of acting steps done
    return f;
}

// launch arguments of k_aggregate_obs (agg_kernels.hip): divided rows in, aggregated rows out
struct AggArgs {
    const int8_t* acc;  // [E][N][C][acc_stride]
    const int8_t* off;  // [E][N][L][off_stride]
    int8_t* out_acc;    // [E][N][agg_acc_stride] or NULL
    int8_t* out_off;    // [E][N][agg_off_stride] or NULL
    int8_t* out_full;   // [E][N][full_stride] or NULL
    int N, C, L, d_acc, acc_stride, off_stride;
    int agg_acc_stride, agg_off_stride, full_stride;
    long long E;
};

// launch arguments of k_regen_agent_rows (agg_kernels.hip)
struct RegenArgs {
    const int8_t* core_rows;   // [M][C][acc_stride]
    const int8_t* core_owner;  // [M][C]
    const int8_t* slot_pairs;  // [M][N][L][2] (offer rows) or NULL
    const int64_t* frame;      // [n] record index
    const int32_t* agent;      // [n] 0-based agent
    int8_t* acc;               // [n][acc_ld] or NULL
    int8_t* off;               // [n][off_ld] or NULL
    long long n;
    int N, C, L, d_acc, acc_stride, acc_ld, off_ld;
};

// Build the record layout and LDS plan for a validated config.
inline Params make_params(const ms_config& c, int32_t cap) {
    Params p{};
    static_cast<Geom&>(p) = make_geom(c.n_agents, c.n_cores, c.collection_length, c.new_jobs_per_round);
    p.K = c.n_kinds;
    p.cap = cap;
    for (int i = 0; i < MS_MAX_KINDS; i++) {
        p.prio[i] = c.job_priority[i];
        p.len[i] = c.job_length[i];
        p.acc[i] = c.acc_probability[i];
        p.fix[i] = c.fix_price[i];
    }
    p.n_fix = c.n_fix_prices;
    p.free_prices = c.free_prices;
    p.commercial = c.commercial_reward;
    p.new_jobs = c.new_jobs_per_round;
    p.mult = c.reward_multiplier;
    p.ep_len = c.episode_length > 0 ? c.episode_length : 1;
    p.net_zero = (float)c.net_zero_offer_reward;
    return p;
}

}  // namespace ms
