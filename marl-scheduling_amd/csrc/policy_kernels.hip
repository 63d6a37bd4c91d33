// policy_kernels.hip — PPO action selection and return estimation for gfx950.
//
// k_act: ActorCritic.act (PPOmodules.py:53-63) for every unit of every env
// replica. A wave takes 16 observation rows at a time and runs
// Linear(D,16)-tanh-Linear(16,16)-tanh-Linear(16,A) with the batch on the MFMA
// column (lane) axis, so each layer's accumulator is the next layer's B operand
// unchanged. Layer 1 is three v_mfma_f32_16x16x32_bf16 per 32 inputs: the int8
// observations are exact in bf16 and the f32 weights are split into three bf16
// terms that sum to them exactly (error of the f32 accumulation only); layers
// 2-3 run on v_mfma_f32_16x16x4_f32 with the weights read in a permuted k order.
// All weights live in registers; the kernel uses no LDS. Softmax, the
// Categorical renormalisation and the inverse-CDF sample run on the accumulator
// layout: a row's logits live in 4 lanes x 4 registers per 16 actions.
// With a second (price) net the kernel is FreePriceOfferPPO.selectAction
// (PPOmodules.py:312-332): core chooser, then the price chooser on
// [obs[2a:2a+2], obs[-2:]] (or the dummy [-5,-5,-5,-5] for a = 0), in one launch.
//
// k_returns: PPO.update's Monte-Carlo returns (PPOmodules.py:128-137) in
// float64, cast to f32 and normalised per sequence.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/marlsched.h"
#include "ms_common.h"
#include "ms_act.h"

#pragma clang fp contract(fast)  // (build.sh: -ffp-contract=fast for this file)

namespace ms {


// Profiling build only (tools/build_act_probe.sh: -DMS_ACT_PROBE): lane 0 of every wave of the paired act
// kernel adds the shader-clock cycles between consecutive marks to a per-(half, phase) counter. The product
// library is built without it and the marks compile to nothing.
#if defined(MS_ACT_PROBE) && (defined(MS_ACT_PAIR_TU) || !defined(MS_SPLIT_PAIR))
#define MS_ACT_PROBE_ON 1
constexpr int kActProbeWaves = 1 << 14;
// per wave slot [half][wave % kActProbeWaves][phase] (plain stores of lane 0: no shared address, so the
// probe's own writes do not queue behind each other in the memory system), summed on the host
__device__ unsigned long long g_act_cycles[2][kActProbeWaves][16];
__device__ unsigned long long g_act_waves[2][kActProbeWaves];
#define MS_AMARK(k)                                                    \
    do {                                                               \
        const uint64_t t_now = __builtin_amdgcn_s_memtime();          \
        t_acc[k] += t_now - t_prev;                                    \
        t_prev = t_now;                                                \
    } while (0)
#define MS_APROBE_BEGIN                                                \
    uint64_t t_prev = __builtin_amdgcn_s_memtime();                    \
    uint64_t t_acc[16] = {};
#define MS_APROBE_END(half)                                            \
    if (lane == 0) {                                                   \
        const int slot = (block * 4 + (threadIdx.x >> 6)) % kActProbeWaves; \
        for (int k = 0; k < 16; k++) g_act_cycles[half][slot][k] += t_acc[k]; \
        g_act_waves[half][slot] += 1ull;                               \
    }
#else
#define MS_AMARK(k) \
    do {            \
    } while (0)
#define MS_APROBE_BEGIN
#define MS_APROBE_END(half)
#endif

struct ActArgs {
    ms_mlp_params n1, n2;  // n2 used only with a price net (NT2 > 0)
    const int8_t* obs;
    int stride, U, S, n_cores;
    int E, n_items;
    int tiles_per_wave, waves_per_group;
    uint64_t seed, offset;
    const uint64_t* offset_dev;
    const float* uniforms;  // [2][E*U] or NULL
    int8_t* action;
    float* logprob;
    int8_t* price_state;   // [E*U][4] (pus = 0) or unit-major: row (e, u) at u * pus + e
    int8_t* price_action;
    float* price_logprob;
    int64_t pus;           // unit stride (rows) of the price chooser's outputs; 0: [E][U]
    int8_t* env_price;
    const int8_t* common;  // [stride] or NULL (k_act_common)
    int items_per_wave;    // k_act_common
    // compact acceptor observations (k_act_common<.., OWN>): obs = core rows [E][C][stride], owner
    // [E][C]; row (e, u = a*C + c) is core row (e, c) if owner[e][c] == a + 1, else the common row
    const int8_t* owner;
    // price chooser sampling table (ms_price_table): ptab [G][pkeys][kPriceTW], pdigit [4][256]
    // (key offset of byte value v at position p, index v + 128; -1: not tabulated); NULL: computed
    const float* ptab;
    const int16_t* pdigit;
    int pkeys;
};

// floats per price-table entry: running sums and log-probs of 16 * NT2 actions, S, last nonzero
template <int NT2>
struct PriceTW {
    static constexpr int v = 32 * NT2 + 4;
};

// One wave = a contiguous range of 16-row tiles of one group; no LDS. Layer 1 runs on the bf16 MFMA
// with the weights split in three bf16 terms (exact f32 weights; the int8 inputs are exact in bf16):
// lane (j, g) loads dwords 8s + 2g, 8s + 2g + 1 of tile row j, which are exactly its B fragment of
// k-step s. S1 = ceil(stride / 32) k-steps.
template <int S1, int NT, int NT2, bool EXT_U>
__device__ __forceinline__ void act_tiles(const ActArgs& a, int block) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int gw = block * 4 + __builtin_amdgcn_readfirstlane(tid >> 6);  // global wave index (wave-uniform)
    const int grp = gw / a.waves_per_group;
    const int wv = gw - grp * a.waves_per_group;
    if (grp >= a.n1.n_groups) return;
    MS_APROBE_BEGIN
    const int j = lane & 15, g4 = lane >> 4;
    constexpr int NP = NT2 > 0 ? NT2 : 1;
    constexpr int TW = PriceTW<NP>::v;
    // the arrays this wave touches as raw buffers (32-bit offsets: row indices < 2^24 and arrays
    // < 2^31 bytes, checked at the launch)
    const long long n_rows = (long long)a.E * a.U;
    const long long n_pc = a.pus ? (long long)a.U * a.pus : n_rows;  // price chooser rows
    const RawBuf obs_b(a.obs, n_rows * a.stride), act_b(a.action, n_rows), lp_b(a.logprob, 4 * n_rows);
    const RawBuf pst_b(a.price_state, 4 * n_pc), pact_b(a.price_action, n_pc), plp_b(a.price_logprob, 4 * n_pc),
        envp_b(a.env_price, n_rows);
    const RawBuf tab_b(a.ptab ? a.ptab + (size_t)grp * a.pkeys * TW : nullptr, 4ll * a.pkeys * TW);
    // the price table's key digits, this wave's copy in LDS (a lookup per row: no memory round trip)
    int16_t* pdig = nullptr;
    if constexpr (NT2 > 0) {
        __shared__ uint32_t s_pd[4][512];
        const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
        if (a.ptab) {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(a.pdigit);
            uint32_t v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) v[k] = src[64 * k + lane];
#pragma unroll
            for (int k = 0; k < 8; k++) s_pd[wid][64 * k + lane] = v[k];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        pdig = reinterpret_cast<int16_t*>(s_pd[wid]);
    }
    W1Split<S1> w1;
    Head<NT> h1;
    if (const uint32_t* fg = frag_groups<S1, NT>(a.n1, false)) {  // made once per weight update
        using FL = FragLayout<S1, NT>;
        const uint32_t* lf = fg + (size_t)grp * FL::GB + lane * FL::LW;
        w1.load_frag(lf);
        h1.load_frag(reinterpret_cast<const float*>(lf + 12 * S1));
    } else {
        w1.load(a.n1.w1 + (size_t)grp * 16 * a.n1.in_dim, a.n1.in_dim, j, g4);
        h1.load(a.n1, grp, j, g4);
    }
    const uint64_t off = a.offset + (a.offset_dev ? *a.offset_dev : 0ull);
    const int stride4 = a.stride >> 2;
    const int n_rows_total = a.E * a.U;
    const int tiles = (a.n_items + 15) >> 4;
    const int t0 = wv * a.tiles_per_wave;
    const int t1 = min(t0 + a.tiles_per_wave, tiles);
    // item i of this group -> obs row: e = i / S by a multiply-high with one correction step
    const uint32_t s_magic = 0xffffffffu / (uint32_t)a.S;
    const uint32_t u_magic = 0xffffffffu / (uint32_t)a.U;  // row -> replica (unit-major price outputs)
    auto row_of_lane = [&](int tile, int jj) -> int {
        const int i = tile * 16 + jj;
        if (i >= a.n_items) return -1;
        int e = (int)__umulhi((uint32_t)i, s_magic);
        if ((e + 1) * a.S <= i) e++;
        return e * a.U + grp * a.S + (i - e * a.S);
    };
    auto row_of = [&](int tile) -> int { return row_of_lane(tile, j); };
    // Philox uniforms, computed for 4 tiles at a time: lane (j, g4) draws for row j of tile
    // base + g4 (counter = the obs row index, so the values do not depend on the tiling)
    uint32_t rnd0 = 0, rnd1 = 0, rb0[4] = {0, 0, 0, 0}, rb1[4] = {0, 0, 0, 0};
    // the counter's row is global across launches (ms_mlp_params.row_base: this call's first replica's
    // first row), so a replica draws the same numbers whichever rank or replica split steps it
    const uint32_t rbase = (uint32_t)a.n1.row_base;
    // With a price net the row's two words are its two uniforms. A single net's row takes word
    // (i >> 6) & 1 of the draw countered by the row of item i & ~64: the rule of k_act_common's scan
    // (one draw per two 64-item steps there), so both kernels sample a row alike.
    auto draw4 = [&](int base) {
        if (NT2 > 0) {
            const int r = base + g4 < t1 ? row_of_lane(base + g4, j) : -1;
            philox2((uint32_t)r + rbase, off, a.seed, rnd0, rnd1);
            rows_bcast(rnd1, rb1);
        } else {
            const int i = (base + g4) * 16 + j;
            const int r = base + g4 < t1 ? row_of_lane(0, i & ~64) : -1;
            philox2((uint32_t)r + rbase, off, a.seed, rnd0, rnd1);
            if (i & 64) rnd0 = rnd1;
        }
        rows_bcast(rnd0, rb0);  // tile base + k takes row k's draws
    };
    auto pick4 = [](const uint32_t (&v)[4], int k) { return k == 0 ? v[0] : (k == 1 ? v[1] : (k == 2 ? v[2] : v[3])); };
    // Two tiles per step: their MFMA chains, transcendentals and memory round trips interleave (the
    // kernel is latency-bound with a few waves per SIMD), and their cross-lane sums pair up. A lone
    // last tile runs beside an empty partner (rows -1: nothing written).
    const int A1 = a.n1.n_actions;
    // the pair's uniforms (Philox for 4 tiles at a time, or the given ones)
    auto uniforms2 = [&](int tile, const int (&cur)[2], float (&u1)[2], float (&u2)[2]) {
        if (EXT_U) {
#pragma unroll
            for (int i = 0; i < 2; i++) {
                u1[i] = cur[i] >= 0 ? a.uniforms[cur[i]] : 0.f;
                u2[i] = cur[i] >= 0 && NT2 > 0 ? a.uniforms[n_rows_total + cur[i]] : 0.f;
            }
        } else {
            const int k = (tile - t0) & 3;  // 0 or 2
            if (k == 0) draw4(tile);
#pragma unroll
            for (int i = 0; i < 2; i++) {
                u1[i] = u24(pick4(rb0, k + i));
                u2[i] = u24(pick4(rb1, k + i));
            }
        }
    };
    // the core chooser (or the only net) of both tiles
    auto core2 = [&](const uint32_t (&xd)[2][S1][2], const float (&u1)[2], int (&act)[2], float (&lp)[2]) {
        f4 acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
        for (int s = 0; s < S1; s++) {
            u4v x[2];
#pragma unroll
            for (int i = 0; i < 2; i++) x[i] = bytes_to_bf16(xd[i][s][0], xd[i][s][1]);
#pragma unroll
            for (int i = 0; i < 2; i++) acc[i] = mfma_bf16(w1.hi[s], x[i], acc[i]);
#pragma unroll
            for (int i = 0; i < 2; i++) acc[i] = mfma_bf16(w1.mid[s], x[i], acc[i]);
#pragma unroll
            for (int i = 0; i < 2; i++) acc[i] = mfma_bf16(w1.lo[s], x[i], acc[i]);
        }
        h1.run2(acc, A1, g4, u1, act, lp);
    };
    // price chooser input (PPOmodules.py:316-327): lane g4 takes row byte k of
    // [obs[2a], obs[2a+1], obs[-2], obs[-1]] (obs[-2:] = the slot's pair at 2C), or -5 for a = 0; and
    // the byte's offset in the price table's key (-1: not tabulated; rows of an empty tile: 0)
    auto price_in2 = [&](const uint32_t (&xd)[2][S1][2], const int (&cur)[2], const int (&act)[2], int (&pin)[2],
                         int (&dg)[2]) {
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int k = g4 < 2 ? 2 * act[i] + g4 : 2 * a.n_cores + (g4 - 2);
            const int src = j + 16 * ((k >> 3) & 3), ks = k >> 5, kh = (k >> 2) & 1;
            uint32_t dw = 0;
#pragma unroll
            for (int s = 0; s < S1; s++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const uint32_t v = (uint32_t)__shfl((int)xd[i][s][h], src);
                    if (s == ks && h == kh) dw = v;
                }
            pin[i] = act[i] == 0 ? -5 : (int)(int8_t)(dw >> (8 * (k & 3)));
            dg[i] = !a.ptab ? -1 : (cur[i] >= 0 ? (int)pdig[g4 * 256 + pin[i] + 128] : 0);
        }
    };
    // the price chooser's outputs of both tiles
    auto price_out2 = [&](const int (&cur)[2], const int (&act)[2], const int (&pin)[2], const int (&pact)[2],
                          const float (&plp)[2]) {
#pragma unroll
        for (int i = 0; i < 2; i++) {
            if (cur[i] >= 0) {
                // the price chooser's rollout rows: [E][U], or unit-major (the update reads one unit's
                // rows of every replica, so they lie contiguous)
                uint32_t pc = (uint32_t)cur[i];
                if (a.pus) {
                    int e = (int)__umulhi((uint32_t)cur[i], u_magic);
                    if ((e + 1) * a.U <= cur[i]) e++;
                    pc = (uint32_t)(cur[i] - e * a.U) * (uint32_t)a.pus + (uint32_t)e;
                }
                pst_b.st8(4 * pc + g4, pin[i]);
                if (g4 == 0) {
                    pact_b.st8(pc, pact[i]);
                    plp_b.stf(4 * pc, plp[i]);
                    envp_b.st8((uint32_t)cur[i], act[i] == 0 ? -5 : pact[i]);
                }
            }
        }
    };
    uint32_t pre[2][S1][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int s = 0; s < S1; s++) pre[i][s][0] = pre[i][s][1] = 0u;
    // unconditional loads from clamped addresses, used as loaded: the rows past the end are never
    // written and the dwords past the row meet zero weights (so the wait lands at the use)
    auto load_rows = [&](int r, uint32_t (&dst)[S1][2]) {
        const uint32_t rb = __umul24((uint32_t)(r < 0 ? 0 : r), (uint32_t)a.stride);
#pragma unroll
        for (int s = 0; s < S1; s++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int cc = 8 * s + 2 * g4 + h;
                dst[s][h] = obs_b.ld32(rb + 4 * (cc < stride4 ? cc : stride4 - 1));
            }
    };
    int row[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
        row[i] = t0 + i < t1 ? row_of(t0 + i) : -1;
        if (t0 + i < t1) load_rows(row[i], pre[i]);
    }
    bool any_miss = false;  // a pair with a price input outside the table: priced after the loop
    MS_AMARK(0);  // setup: weights / fragments, the price digits, the first rows' loads issued
    for (int tile = t0; tile < t1; tile += 2) {
        uint32_t xd[2][S1][2];
        int cur[2];
#pragma unroll
        for (int i = 0; i < 2; i++) {
#pragma unroll
            for (int s = 0; s < S1; s++) xd[i][s][0] = pre[i][s][0], xd[i][s][1] = pre[i][s][1];
            cur[i] = row[i];
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            row[i] = tile + 2 + i < t1 ? row_of(tile + 2 + i) : -1;
            if (tile + 2 + i < t1) load_rows(row[i], pre[i]);
        }
        MS_AMARK(1);  // row indices + the next pair's loads issued
        float u1[2], u2[2];
        uniforms2(tile, cur, u1, u2);
        MS_AMARK(2);  // Philox
        int act[2];
        float lp[2];
        core2(xd, u1, act, lp);
        MS_AMARK(3);  // core chooser (layer 1 waits for this pair's rows)
        if (NT2 > 0) {
            int pin[2], dg[2];
            price_in2(xd, cur, act, pin, dg);
            if (a.ptab && __ballot(dg[0] < 0 || dg[1] < 0) == 0ull) {
                // every row of both tiles is tabulated: sample from the table (Head::run's arithmetic)
                rows_sum2_i(dg[0], dg[1]);
                float cum[2][NP][4], S2[2];
                int lnz[2], cnt[2], pact[2];
                float plp[2];
                uint32_t te[2];  // byte offset of the row's table entry
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    te[i] = __umul24((uint32_t)dg[i], 4u * TW);
#pragma unroll
                    for (int t = 0; t < NP; t++) {
                        const auto c4 = __builtin_amdgcn_raw_buffer_load_b128(tab_b.r, (int)(te[i] + 4 * (16 * t + 4 * g4)), 0, 0);
#pragma unroll
                        for (int q = 0; q < 4; q++) cum[i][t][q] = __uint_as_float(c4[q]);
                    }
                    S2[i] = tab_b.ldf(te[i] + 4 * (32 * NP));
                    lnz[i] = (int)tab_b.ld32(te[i] + 4 * (32 * NP + 1));
                }
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const float target = u2[i] * S2[i];
                    cnt[i] = 0;
#pragma unroll
                    for (int t = 0; t < NP; t++)
#pragma unroll
                        for (int q = 0; q < 4; q++) cnt[i] += (cum[i][t][q] <= target) ? 1 : 0;
                }
                rows_sum2_i(cnt[0], cnt[1]);
                // the chosen action's log-prob straight from its table entry (one load per row)
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    pact[i] = cnt[i] >= a.n2.n_actions ? lnz[i] : cnt[i];
                    plp[i] = tab_b.ldf(te[i] + 4 * (16 * NP + pact[i]));
                }
                price_out2(cur, act, pin, pact, plp);
            } else {
                any_miss = true;
            }
        }
        MS_AMARK(4);  // price chooser: input, table entry, sample, its stores
#pragma unroll
        for (int i = 0; i < 2; i++)
            if (cur[i] >= 0 && g4 == 0) {
                act_b.st8((uint32_t)cur[i], act[i]);
                lp_b.stf(4 * (uint32_t)cur[i], lp[i]);
            }
        MS_AMARK(5);  // core chooser stores
    }
    if (NT2 > 0 && any_miss) {
        // the pairs the table could not serve (or every pair, without a table): the same pairs and
        // draws again, the core chooser recomputed (bit-identical), then the price net itself; its
        // weights take registers only here, after the main loop
        Head<NP> h2;
        h2.load(a.n2, grp, j, g4);
        const float pw1 = a.n2.w1[((size_t)grp * 16 + j) * 4 + g4];  // W1p[j][g4] (K = 4 inputs)
        for (int tile = t0; tile < t1; tile += 2) {
            uint32_t xd[2][S1][2];
            int cur[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                cur[i] = tile + i < t1 ? row_of(tile + i) : -1;
                load_rows(cur[i], xd[i]);
            }
            float u1[2], u2[2];
            uniforms2(tile, cur, u1, u2);
            int act[2], pin[2], dg[2];
            float lp[2];
            core2(xd, u1, act, lp);
            price_in2(xd, cur, act, pin, dg);
            if (a.ptab && __ballot(dg[0] < 0 || dg[1] < 0) == 0ull) continue;  // priced in the main loop
            int pact[2];
            float plp[2];
            f4 acc2[2];
#pragma unroll
            for (int i = 0; i < 2; i++) acc2[i] = mfma4(pw1, (float)pin[i], (f4){0, 0, 0, 0});
            h2.run2(acc2, a.n2.n_actions, g4, u2, pact, plp);
            price_out2(cur, act, pin, pact, plp);
        }
    }
    MS_AMARK(6);  // untabulated price inputs
    MS_APROBE_END(0)
}

// ---------------------------------------------------------------------------
// k_act_common: ActorCritic.act where many rows equal one common row. Acceptor observations are
// mostly the constant row [0, -1, -1, (-2, -2) * O] of a core the agent does not own
// (Agent.py:167-212: no own job, and every offer to the core is addressed to its owner), so the
// network output of those rows is the same: the wave computes the common row's sampling table
// once (Head::table, the exact arithmetic of Head::run) and samples each row equal to it from its
// own uniform with a handful of compares. The other rows are collected in LDS and run through the
// MFMA tiles as in k_act. Outputs are bit-identical to k_act's.
#ifndef MS_COMMON_SEG
#define MS_COMMON_SEG 512
#endif
constexpr int kCommonSeg = MS_COMMON_SEG;  // most rows per wave = capacity of the wave's LDS row list

template <int S1, int NT, int NT2, bool EXT_U>
__global__ void __launch_bounds__(256) k_act(ActArgs a) {
    act_tiles<S1, NT, NT2, EXT_U>(a, blockIdx.x);
}

template <int S1, int NT, bool EXT_U, bool OWN>
__device__ __forceinline__ void act_common_rows(const ActArgs& a, int block) {
    __shared__ int32_t s_list[4][kCommonSeg];
    __shared__ float s_ulist[4][kCommonSeg];  // the listed rows' uniforms (drawn in the scan)
    __shared__ float s_cum[4][16 * NT], s_lp[4][16 * NT], s_S[4];
    __shared__ int s_lnz[4];
    __shared__ uint32_t s_tmpl[4][8 * S1];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int gw = block * 4 + wid;
    const int grp = gw / a.waves_per_group;
    const int wv = gw - grp * a.waves_per_group;
    if (grp >= a.n1.n_groups) return;  // whole waves only: the kernel has no block barrier
    MS_APROBE_BEGIN
    const int j = lane & 15, g4 = lane >> 4;
    const int A = a.n1.n_actions;
    const int stride4 = a.stride >> 2;
    W1Split<S1> w1;
    Head<NT> h1;
    if (const uint32_t* fg = frag_groups<S1, NT>(a.n1, true)) {
        // the weights and the common row's sampling table as ms_act_prepare made them
        using FL = FragLayout<S1, NT>;
        const uint32_t* gb = fg + (size_t)grp * FL::GB;
        w1.load_frag(gb + lane * FL::LW);
        h1.load_frag(reinterpret_cast<const float*>(gb + lane * FL::LW + 12 * S1));
        const uint32_t* tb = gb + 64 * FL::LW;
        for (int k = lane; k < 32 * NT + 2; k += 64) {
            const uint32_t v = tb[k];
            if (k < 16 * NT)
                s_cum[wid][k] = __uint_as_float(v);
            else if (k < 32 * NT)
                s_lp[wid][k - 16 * NT] = __uint_as_float(v);
            else if (k == 32 * NT)
                s_S[wid] = __uint_as_float(v);
            else
                s_lnz[wid] = (int)v;
        }
    } else {
        w1.load(a.n1.w1 + (size_t)grp * 16 * a.n1.in_dim, a.n1.in_dim, j, g4);
        h1.load(a.n1, grp, j, g4);
        common_table<S1, NT>(w1, h1, a.common, stride4, s_tmpl[wid], s_cum[wid], s_lp[wid], &s_S[wid], &s_lnz[wid],
                             lane);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t off = a.offset + (a.offset_dev ? *a.offset_dev : 0ull);
    int32_t* list = s_list[wid];
    float* ulist = s_ulist[wid];
    const uint32_t* crow = reinterpret_cast<const uint32_t*>(a.common);
    const float* cum = s_cum[wid];  // the running sums, non-decreasing (z >= 0): binary-searched in LDS
    constexpr int LPR = S1 <= 2 ? 4 : (S1 <= 4 ? 8 : 16);
    CommonScan<LPR> cs;
    if (!OWN) cs.init(crow, stride4, lane);
    const float S = s_S[wid];
    const int last_nz = s_lnz[wid];
    const uint32_t s_magic = 0xffffffffu / (uint32_t)a.S;
    auto row_of_item = [&](int i) -> int {
        int e = (int)__umulhi((uint32_t)i, s_magic);
        if ((e + 1) * a.S <= i) e++;
        return e * a.U + grp * a.S + (i - e * a.S);
    };
    // the outputs as raw buffers: 32-bit row offsets, no 64-bit address arithmetic per store
    // (act_common_fits: E * U * 4 bytes < 2^31)
    const long long n_rows = (long long)a.E * a.U;
    const RawBuf act_b(a.action, n_rows), lp_b(a.logprob, 4 * n_rows);
    const int i_begin = wv * a.items_per_wave;
    const int i_end = min(i_begin + a.items_per_wave, a.n_items);  // <= kCommonSeg rows
    // Item i's uniform: word (i >> 6) & 1 of the Philox draw countered by the row of item i & ~64, so
    // one draw serves the rows of two 64-item scan steps (the second step reuses the first's other
    // word). A function of the item index alone: the same for any split of the items into waves.
    uint32_t u_other = 0;  // the draw's second word, kept from the first step of the pair
    auto step_uniform = [&](int i0, int row) -> float {  // i0 = the step's first item (multiple of 64)
        if (EXT_U) return a.uniforms[row < 0 ? 0 : row];
        if ((i0 & 64) && i0 > i_begin) return u24(u_other);
        const int ib = (i0 & ~64) + lane;
        uint32_t r0, r1;
        philox2((uint32_t)row_of_item(ib) + (uint32_t)a.n1.row_base, off, a.seed, r0, r1);
        u_other = r1;
        return u24((i0 & 64) ? r1 : r0);
    };
    const uint64_t below = (1ull << lane) - 1ull;
    int n_list = 0;
    // ---- scan (one 64-row step ahead in registers): rows equal to the common row are sampled
    //      from the table, the others listed
    int n_row = 0;
    bool n_in = false;
    // compact rows: the core row of (e, u) and whether agent u / C + 1 owns core u % C
    // (quotients by a multiply-high with one correction step, as row_of_item: no per-row
    // integer-division sequence)
    const uint32_t u_mag = 0xffffffffu / (uint32_t)a.U, c_mag = 0xffffffffu / (uint32_t)a.n_cores;
    auto core_row_of = [&](int row, int& c_out) -> size_t {
        int e = (int)__umulhi((uint32_t)row, u_mag);
        if ((e + 1) * a.U <= row) e++;
        const int u = row - e * a.U;
        int ag = (int)__umulhi((uint32_t)u, c_mag);
        if ((ag + 1) * a.n_cores <= u) ag++;
        c_out = ag;
        return (size_t)e * a.n_cores + (u - ag * a.n_cores);
    };
    auto load_step = [&](int i0) {
        if constexpr (!OWN) {
            cs.load([&](int k) {
                const int i = i0 + k;
                return reinterpret_cast<const uint32_t*>(a.obs + (size_t)(i < i_end ? row_of_item(i) : 0) * a.stride);
            }, lane);
        }
        const int i = i0 + lane;
        n_in = i < i_end;
        n_row = n_in ? row_of_item(i) : 0;
    };
    // one 64-row step: common rows sample from the table, the others are listed
    auto scan_step = [&](int i0, int row, bool in, bool common) {
        // every lane draws (the lanes of listed rows keep theirs for the tile pass: no second draw
        // there, and no lane-group-replicated one)
        MS_AMARK(2);  // (scan bookkeeping)
        const float u = step_uniform(i0, row);
        MS_AMARK(3);  // Philox (every other step)
        if (common) {
            const float target = u * S;
            // the number of running sums <= target (Head::run's count), by binary search
            int cnt = 0;
#pragma unroll
            for (int step = 16 * NT; step >= 1; step >>= 1)
                if (cnt + step <= 16 * NT && cum[cnt + step - 1] <= target) cnt += step;
            const int act = cnt >= A ? last_nz : cnt;
            act_b.st8((uint32_t)row, act);
            lp_b.stf(4 * (uint32_t)row, s_lp[wid][act]);
        }
        const bool other = in && !common;
        const uint64_t m = __ballot(other);
        if (other) {
            list[n_list + __popcll(m & below)] = row;
            ulist[n_list + __popcll(m & below)] = u;
        }
        n_list += __popcll(m);
        MS_AMARK(4);  // table search, stores, row list
    };
    MS_AMARK(0);  // setup: fragments, the common row's table
    if constexpr (OWN) {
        // compact rows: every step's owner byte is loaded up front (one memory round trip per wave)
        constexpr int MS = kCommonSeg / 64;
        int8_t own_st[MS], me_st[MS];
        int row_st[MS];
        // a group of exactly one agent's C acceptors (locally shared: S == C, unit a*C + c): item i of
        // group g is core row i (replica i / C, core i % C) and the agent is g, so the core row and the
        // owner byte need no per-item quotient
        const bool agent_group = a.S == a.n_cores;
        const RawBuf own_b(a.owner, (long long)a.E * a.n_cores);
#pragma unroll
        for (int st = 0; st < MS; st++) {
            const int i = i_begin + 64 * st + lane;
            row_st[st] = i < i_end ? row_of_item(i) : -1;
            if (agent_group) {
                own_st[st] = (int8_t)own_b.ld8s((uint32_t)(i < i_end ? i : 0));
                me_st[st] = (int8_t)(grp + 1);
            } else {
                int ag;
                const size_t cr = core_row_of(row_st[st] < 0 ? 0 : row_st[st], ag);
                own_st[st] = a.owner[cr];
                me_st[st] = (int8_t)(ag + 1);
            }
        }
        MS_AMARK(1);  // owner loads issued
#pragma unroll
        for (int st = 0; st < MS; st++)
            if (i_begin + 64 * st < i_end)
                scan_step(i_begin + 64 * st, row_st[st], row_st[st] >= 0, row_st[st] >= 0 && own_st[st] != me_st[st]);
    } else {
        // (one 64-row step ahead in registers)
        if (i_begin < i_end) load_step(i_begin);
        for (int i0 = i_begin; i0 < i_end; i0 += 64) {
            const int row = n_row;
            const bool in = n_in;
            const bool common = cs.lane_row_common(lane) && in;
            if (i0 + 64 < i_end) load_step(i0 + 64);
            scan_step(i0, row, in, common);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- the listed rows in 16-row MFMA tiles, two tiles per step (k_act's path; the next pair's rows
    //      prefetched, a lone last tile beside an empty partner)
    uint32_t tp[2][S1][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int s = 0; s < S1; s++) tp[i][s][0] = tp[i][s][1] = 0u;
    int t_row[2] = {-1, -1};
    float t_u[2] = {0.f, 0.f};
    auto load_tile = [&](int i, int t0) {  // tile starting at list entry t0 (< n_list)
        const int k = t0 + j < n_list ? t0 + j : t0;
        t_row[i] = t0 + j < n_list ? list[k] : -1;
        t_u[i] = ulist[k];
        size_t sr = (size_t)list[k];
        if constexpr (OWN) {
            int ag;
            sr = core_row_of(list[k], ag);
        }
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.obs + sr * a.stride);
#pragma unroll
        for (int s = 0; s < S1; s++) {
            const int c0 = 8 * s + 2 * g4;
            tp[i][s][0] = src[c0 < stride4 ? c0 : stride4 - 1];
            tp[i][s][1] = src[c0 + 1 < stride4 ? c0 + 1 : stride4 - 1];
        }
    };
#pragma unroll
    for (int i = 0; i < 2; i++)
        if (16 * i < n_list) load_tile(i, 16 * i);
    MS_AMARK(5);  // list barrier + first tiles' loads issued
    for (int t0 = 0; t0 < n_list; t0 += 32) {
        int row[2];
        float u[2];
        f4 acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
        for (int s = 0; s < S1; s++) {
            u4v x[2];
#pragma unroll
            for (int i = 0; i < 2; i++) x[i] = bytes_to_bf16(tp[i][s][0], tp[i][s][1]);
#pragma unroll
            for (int i = 0; i < 2; i++) acc[i] = mfma_bf16(w1.hi[s], x[i], acc[i]);
#pragma unroll
            for (int i = 0; i < 2; i++) acc[i] = mfma_bf16(w1.mid[s], x[i], acc[i]);
#pragma unroll
            for (int i = 0; i < 2; i++) acc[i] = mfma_bf16(w1.lo[s], x[i], acc[i]);
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            row[i] = t0 + 16 * i < n_list ? t_row[i] : -1;
            u[i] = t_u[i];
            if (t0 + 32 + 16 * i < n_list) load_tile(i, t0 + 32 + 16 * i);
        }
        MS_AMARK(6);  // listed rows: layer 1 (waits for their loads), the next pair's loads issued
        int act[2];
        float lp[2];
        h1.run2(acc, A, g4, u, act, lp);
        MS_AMARK(7);  // listed rows: layers 2-3, softmax, sample
#pragma unroll
        for (int i = 0; i < 2; i++)
            if (row[i] >= 0 && g4 == 0) {
                act_b.st8((uint32_t)row[i], act[i]);
                lp_b.stf(4 * (uint32_t)row[i], lp[i]);
            }
        MS_AMARK(8);  // listed rows' stores
    }
    MS_APROBE_END(1)
}

// launch-shape knobs for measurements (tools/); the defaults are the measured best for cfg3
static long long env_int(const char* name, long long dflt) {
    const char* v = getenv(name);
    return v && *v ? atoll(v) : dflt;
}

template <int S1, int NT, bool EXT_U, bool OWN>
__global__ void __launch_bounds__(256) k_act_common(ActArgs a) {
    act_common_rows<S1, NT, EXT_U, OWN>(a, blockIdx.x);
}

// getActionForAllAgents of a free-price round (SchedulingEnvironment.py:150-172) in one launch: the
// first off_blocks blocks run the offer units (core + price chooser, k_act), the rest the acceptor
// units on compact rows (k_act_common). The two workloads' waves share the CUs, so one's waits
// hide under the other's work instead of each launch waiting out its own chain.
// (four 4-wave blocks per CU; two for cfg4's acceptor half, whose 128-input rows and 64 action slots take
// ~250 registers)
#ifndef MS_ACT_PAIR_MINB
#define MS_ACT_PAIR_MINB 4
#endif
template <int S1a, int NTa, int NT2a, int S1b, int NTb>
__global__ void __launch_bounds__(256, (S1b >= 4 ? 2 : MS_ACT_PAIR_MINB)) k_act_pair(ActArgs off, ActArgs acc, int off_blocks) {
    if ((int)blockIdx.x < off_blocks)
        act_tiles<S1a, NTa, NT2a, false>(off, blockIdx.x);
    else
        act_common_rows<S1b, NTb, false, true>(acc, (int)blockIdx.x - off_blocks);
}

// launch shapes (set the wave split in a, return the blocks)
static unsigned act_common_blocks(ActArgs& a, long long target) {
    const int G = a.n1.n_groups;
    // ~target waves over all groups, whole 64-row scan steps each, at most one LDS list of rows
    long long ipw = ((long long)a.n_items * G + target - 1) / target;
    ipw = (ipw + 127) / 128 * 128;  // whole step pairs (one Philox draw serves two steps)
    ipw = ipw < 128 ? 128 : (ipw > kCommonSeg ? kCommonSeg : ipw);
    a.items_per_wave = (int)ipw;
    a.waves_per_group = (a.n_items + a.items_per_wave - 1) / a.items_per_wave;
    const long long waves = (long long)a.waves_per_group * G;
    return (unsigned)((waves + 3) / 4);
}

// act_common_rows stores through 31-bit byte offsets (RawBuf) and reads compact owners by item index
static bool act_common_fits(const ActArgs& a) {
    return (long long)a.E * a.U * 4 <= 0x7fffffffll && (long long)a.E * (a.n_cores > 0 ? a.n_cores : 1) <= 0x7fffffffll;
}

template <int S1, int NT>
static hipError_t launch_act_common_t(ActArgs& a, hipStream_t st) {
    if (!act_common_fits(a)) return hipErrorInvalidValue;
    auto kern = a.owner ? (a.uniforms ? k_act_common<S1, NT, true, true> : k_act_common<S1, NT, false, true>)
                        : (a.uniforms ? k_act_common<S1, NT, true, false> : k_act_common<S1, NT, false, false>);
    static const long long target = env_int("MS_ACT_COMMON_WAVES", 1536);  // measured best for cfg3 alone
    const unsigned blocks = act_common_blocks(a, target);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, st, a);
    return hipGetLastError();
}

// act_tiles addresses rows with 24-bit row indices and 31-bit byte offsets (RawBuf)
static bool act_tiles_fits(const ActArgs& a) {
    const long long rows = (long long)a.E * a.U;
    const long long pc = a.pus ? (long long)a.U * a.pus : rows;
    return rows < (1ll << 24) && rows * a.stride <= 0x7fffffffll && 4 * pc <= 0x7fffffffll &&
           (long long)a.pkeys * PriceTW<8>::v * 4 <= 0x7fffffffll;
}

static unsigned act_blocks(ActArgs& a, long long target) {
    const int G = a.n1.n_groups;
    const int tiles = (a.n_items + 15) / 16;
    // ~target waves over all groups; each wave walks a contiguous tile range with a register prefetch
    int tpw = (int)(((long long)tiles * G + target - 1) / target);
    a.tiles_per_wave = tpw < 1 ? 1 : tpw;
    a.waves_per_group = (tiles + a.tiles_per_wave - 1) / a.tiles_per_wave;
    const long long waves = (long long)a.waves_per_group * G;
    return (unsigned)((waves + 3) / 4);
}

template <int S1, int NT, int NT2>
static hipError_t launch_act_t(ActArgs& a, hipStream_t st) {
    if (!act_tiles_fits(a)) return hipErrorInvalidValue;
    auto kern = a.uniforms ? k_act<S1, NT, NT2, true> : k_act<S1, NT, NT2, false>;
    static const long long target = env_int("MS_ACT_WAVES", 8192);  // measured best for cfg3 alone
    const unsigned blocks = act_blocks(a, target);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, st, a);
    return hipGetLastError();
}

template <int S1>
static hipError_t dispatch_act_s(ActArgs& a, hipStream_t st) {
    const int nt = (a.n1.n_actions + 15) / 16;
    const int nt2 = a.n2.n_groups > 0 ? (a.n2.n_actions + 15) / 16 : 0;
#define MS_ACT(T, T2) \
    if (nt <= T && nt2 == T2) return launch_act_t<S1, T, T2>(a, st);
    if (a.common && a.stride >= 16) {
        if (nt2 != 0) return hipErrorInvalidValue;
        if (nt <= 1) return launch_act_common_t<S1, 1>(a, st);
        if (nt <= 2) return launch_act_common_t<S1, 2>(a, st);
        if (nt <= 4) return launch_act_common_t<S1, 4>(a, st);
        return launch_act_common_t<S1, 8>(a, st);
    }
    if (nt2 == 0) {
        MS_ACT(1, 0) MS_ACT(2, 0) MS_ACT(4, 0) MS_ACT(8, 0)
    } else if (nt2 == 1) {
        MS_ACT(1, 1) MS_ACT(2, 1) MS_ACT(4, 1)
    } else if (nt2 == 2) {
        MS_ACT(1, 2) MS_ACT(2, 2) MS_ACT(4, 2)
    } else if (nt2 <= 8) {
        if (nt <= 4) return launch_act_t<S1, 4, 8>(a, st);
    }
#undef MS_ACT
    return hipErrorInvalidValue;
}

static hipError_t dispatch_act(ActArgs& a, hipStream_t st) {
    const int s1 = (a.stride + 31) / 32;
    if (a.n2.n_groups > 0 && a.n2.in_dim != 4) return hipErrorInvalidValue;
    if (s1 <= 1) return dispatch_act_s<1>(a, st);
    if (s1 <= 2) return dispatch_act_s<2>(a, st);
    if (s1 <= 4) return dispatch_act_s<4>(a, st);
    if (s1 <= 8) return dispatch_act_s<8>(a, st);
    return hipErrorInvalidValue;
}

#ifndef MS_ACT_PAIR_TU  // (the paired act kernel's translation unit defines only launch_act_round)
hipError_t launch_policy_act(const ms_mlp_params* p, const int8_t* obs, int stride, int64_t E, int U, int S,
                             const int8_t* common, uint64_t seed, uint64_t offset, const uint64_t* offset_dev,
                             const float* uniforms, int8_t* action, float* logprob, hipStream_t st) {
    ActArgs a{};
    a.common = common;
    a.n1 = *p;
    a.n2.n_groups = 0;
    a.obs = obs;
    a.stride = stride;
    a.U = U;
    a.S = S;
    a.E = (int)E;
    a.n_items = (int)(E * S);
    a.seed = seed;
    a.offset = offset;
    a.offset_dev = offset_dev;
    a.uniforms = uniforms;
    a.action = action;
    a.logprob = logprob;
    return dispatch_act(a, st);
}
#endif

static ActArgs compact_args(const ms_mlp_params* p, const int8_t* core_rows, const int8_t* core_owner, int stride,
                            int64_t E, int U, int S, int n_cores, const int8_t* common, uint64_t seed, uint64_t offset,
                            const uint64_t* offset_dev, const float* uniforms, int8_t* action, float* logprob) {
    ActArgs a{};
    a.common = common;
    a.owner = core_owner;
    a.n_cores = n_cores;
    a.n1 = *p;
    a.n2.n_groups = 0;
    a.obs = core_rows;
    a.stride = stride;
    a.U = U;
    a.S = S;
    a.E = (int)E;
    a.n_items = (int)(E * S);
    a.seed = seed;
    a.offset = offset;
    a.offset_dev = offset_dev;
    a.uniforms = uniforms;
    a.action = action;
    a.logprob = logprob;
    return a;
}

#ifndef MS_ACT_PAIR_TU  // (the paired act kernel's translation unit defines only launch_act_round)
hipError_t launch_policy_act_compact(const ms_mlp_params* p, const int8_t* core_rows, const int8_t* core_owner,
                                     int stride, int64_t E, int U, int S, int n_cores, const int8_t* common,
                                     uint64_t seed, uint64_t offset, const uint64_t* offset_dev, const float* uniforms,
                                     int8_t* action, float* logprob, hipStream_t st) {
    if (!common || stride < 16 || n_cores < 1 || U % n_cores != 0) return hipErrorInvalidValue;
    ActArgs a = compact_args(p, core_rows, core_owner, stride, E, U, S, n_cores, common, seed, offset, offset_dev,
                             uniforms, action, logprob);
    return dispatch_act(a, st);
}
#endif

static ActArgs offer_free_args(const ms_mlp_params* core, const ms_mlp_params* price, const int8_t* obs, int stride,
                               int64_t E, int U, int S, int n_cores, uint64_t seed, uint64_t offset,
                               const uint64_t* offset_dev, const float* uniforms, int8_t* core_action,
                               float* core_logprob, int8_t* price_state, int8_t* price_action, float* price_logprob,
                               int8_t* env_price, int64_t pus) {
    ActArgs a{};
    a.n1 = *core;
    a.n2 = *price;
    a.obs = obs;
    a.stride = stride;
    a.U = U;
    a.S = S;
    a.n_cores = n_cores;
    a.E = (int)E;
    a.n_items = (int)(E * S);
    a.seed = seed;
    a.offset = offset;
    a.offset_dev = offset_dev;
    a.uniforms = uniforms;
    a.action = core_action;
    a.logprob = core_logprob;
    a.price_state = price_state;
    a.price_action = price_action;
    a.price_logprob = price_logprob;
    a.env_price = env_price;
    a.pus = pus;
    return a;
}

#ifndef MS_ACT_PAIR_TU  // (the paired act kernel's translation unit defines only launch_act_round)
hipError_t launch_offer_act_free(const ms_mlp_params* core, const ms_mlp_params* price, const int8_t* obs, int stride,
                                 int64_t E, int U, int S, int n_cores, uint64_t seed, uint64_t offset,
                                 const uint64_t* offset_dev, const float* uniforms, int8_t* core_action,
                                 float* core_logprob, int8_t* price_state, int8_t* price_action, float* price_logprob,
                                 int8_t* env_price, int64_t pus, hipStream_t st) {
    ActArgs a = offer_free_args(core, price, obs, stride, E, U, S, n_cores, seed, offset, offset_dev, uniforms,
                                core_action, core_logprob, price_state, price_action, price_logprob, env_price, pus);
    return dispatch_act(a, st);
}
#endif

// ms_act_prepare: one wave per group writes each lane's fragment (what the acting waves would derive:
// W1Split::load, Head::load) and, with a common row, its sampling table (common_table: the same
// arithmetic as the acting waves', so acting with the block is bit-identical to acting without).
template <int S1, int NT>
__global__ void __launch_bounds__(64) k_act_prep(ms_mlp_params p, const int8_t* common, int stride, uint32_t* frag) {
    using FL = FragLayout<S1, NT>;
    __shared__ uint32_t tmpl[8 * S1];
    __shared__ float cum[16 * NT], lp[16 * NT], S;
    __shared__ int lnz;
    const int grp = blockIdx.x, lane = threadIdx.x, j = lane & 15, g4 = lane >> 4;
    W1Split<S1> w1;
    w1.load(p.w1 + (size_t)grp * 16 * p.in_dim, p.in_dim, j, g4);
    Head<NT> h1;
    h1.load(p, grp, j, g4);
    uint32_t* gb = frag + 4 + (size_t)grp * FL::GB;
    w1.store_frag(gb + lane * FL::LW);
    h1.store_frag(reinterpret_cast<float*>(gb + lane * FL::LW + 12 * S1));
    if (common) {
        common_table<S1, NT>(w1, h1, common, stride >> 2, tmpl, cum, lp, &S, &lnz, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t* tb = gb + 64 * FL::LW;
        for (int k = lane; k < FL::TB; k += 64)
            tb[k] = k < 16 * NT ? __float_as_uint(cum[k])
                                : (k < 32 * NT ? __float_as_uint(lp[k - 16 * NT])
                                               : (k == 32 * NT ? __float_as_uint(S) : (k == 32 * NT + 1 ? (uint32_t)lnz : 0u)));
    }
    if (grp == 0 && lane < 4)
        frag[lane] = lane == 0 ? kFragMagic : (lane == 1 ? (uint32_t)S1 : (lane == 2 ? (uint32_t)NT : (common ? 1u : 0u)));
}

static bool act_frag_shape(int stride, int A, int& s1, int& nt) {
    s1 = (stride + 31) / 32;
    s1 = s1 <= 1 ? 1 : (s1 <= 2 ? 2 : (s1 <= 4 ? 4 : (s1 <= 8 ? 8 : 0)));
    nt = (A + 15) / 16;
    nt = nt <= 1 ? 1 : (nt <= 2 ? 2 : (nt <= 4 ? 4 : (nt <= 8 ? 8 : 0)));
    return s1 > 0 && nt > 0;
}

#ifndef MS_ACT_PAIR_TU  // (the paired act kernel's translation unit defines only launch_act_round)
size_t act_frag_bytes(const ms_mlp_params* p, int stride) {
    int s1, nt;
    if (!act_frag_shape(stride, p->n_actions, s1, nt)) return 0;
    const int lw = 12 * s1 + 12 + 8 * nt, gb = 64 * lw + 32 * nt + 4;
    return 4 * (4 + (size_t)p->n_groups * gb);
}
#endif

template <int S1>
static hipError_t launch_act_prep_s(const ms_mlp_params* p, const int8_t* common, int stride, uint32_t* frag, int nt,
                                    hipStream_t st) {
    const dim3 grid((unsigned)p->n_groups);
    switch (nt) {
        case 1: hipLaunchKernelGGL((k_act_prep<S1, 1>), grid, dim3(64), 0, st, *p, common, stride, frag); break;
        case 2: hipLaunchKernelGGL((k_act_prep<S1, 2>), grid, dim3(64), 0, st, *p, common, stride, frag); break;
        case 4: hipLaunchKernelGGL((k_act_prep<S1, 4>), grid, dim3(64), 0, st, *p, common, stride, frag); break;
        default: hipLaunchKernelGGL((k_act_prep<S1, 8>), grid, dim3(64), 0, st, *p, common, stride, frag); break;
    }
    return hipGetLastError();
}

#ifndef MS_ACT_PAIR_TU  // (the paired act kernel's translation unit defines only launch_act_round)
hipError_t launch_act_prepare(const ms_mlp_params* p, const int8_t* common, int stride, void* frag, hipStream_t st) {
    int s1, nt;
    if (!act_frag_shape(stride, p->n_actions, s1, nt) || p->hidden != 16) return hipErrorInvalidValue;
    uint32_t* f = static_cast<uint32_t*>(frag);
    switch (s1) {
        case 1: return launch_act_prep_s<1>(p, common, stride, f, nt, st);
        case 2: return launch_act_prep_s<2>(p, common, stride, f, nt, st);
        case 4: return launch_act_prep_s<4>(p, common, stride, f, nt, st);
        default: return launch_act_prep_s<8>(p, common, stride, f, nt, st);
    }
}
#endif

// The price chooser's sampling table (ms_price_table_build): the forward of every tabulated 4-byte
// input per group (16 keys per tile, one per column), stored as Head::run would use it.
template <int NT2>
__global__ void __launch_bounds__(256) k_price_table(ms_mlp_params pn, const int8_t* rows, int K, float* tab) {
    constexpr int TW = PriceTW<NT2>::v;
    const int tid = threadIdx.x, lane = tid & 63, j = lane & 15, g4 = lane >> 4;
    const int gw = blockIdx.x * 4 + (tid >> 6);
    const int tiles = (K + 15) / 16;
    const int grp = gw / tiles, tile = gw - grp * tiles;
    if (grp >= pn.n_groups) return;
    Head<NT2> h;
    h.load(pn, grp, j, g4);
    const float pw1 = pn.w1[((size_t)grp * 16 + j) * 4 + g4];
    const int key = 16 * tile + j;
    const int8_t pin = rows[(size_t)min(key, K - 1) * 4 + g4];
    f4 acc = {0, 0, 0, 0};
    acc = mfma4(pw1, (float)pin, acc);
    float c[NT2][4], lp[NT2][4], S;
    int lnz;
    h.row_table(acc, j, g4, c, lp, S, lnz);
    if (key < K) {
        float* te = tab + ((size_t)grp * K + key) * TW;
#pragma unroll
        for (int t = 0; t < NT2; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                te[16 * t + 4 * g4 + q] = c[t][q];
                te[16 * NT2 + 16 * t + 4 * g4 + q] = lp[t][q];
            }
        if (g4 == 0) {
            te[32 * NT2] = S;
            te[32 * NT2 + 1] = __int_as_float(lnz);
        }
    }
}

#ifndef MS_ACT_PAIR_TU  // (the paired act kernel's translation unit defines only launch_act_round)
hipError_t launch_price_table(const ms_mlp_params* pn, const int8_t* rows, int K, float* tab, hipStream_t st) {
    if (pn->in_dim != 4 || pn->hidden != 16 || K < 1) return hipErrorInvalidValue;
    const int nt = (pn->n_actions + 15) / 16;
    const long long waves = (long long)pn->n_groups * ((K + 15) / 16);
    const dim3 grid((unsigned)((waves + 3) / 4));
    if (nt <= 1)
        hipLaunchKernelGGL(k_price_table<1>, grid, dim3(256), 0, st, *pn, rows, K, tab);
    else if (nt <= 2)
        hipLaunchKernelGGL(k_price_table<2>, grid, dim3(256), 0, st, *pn, rows, K, tab);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}
#endif

// both halves of a free-price round's acting in one launch when their shapes have a paired kernel
// (cfg3: offer rows of <= 32 bytes, <= 16 actions; acceptor rows of <= 64 bytes, <= 32 actions),
// else the two launches in order
#if !defined(MS_SPLIT_PAIR) || defined(MS_ACT_PAIR_TU)  // act_pair_kernels.hip (build.sh)
hipError_t launch_act_round(const ms_mlp_params* core, const ms_mlp_params* price, const int8_t* off_obs,
                            int off_stride, int off_U, int off_S, const ms_mlp_params* acc,
                            const int8_t* core_rows, const int8_t* core_owner, int acc_stride, int acc_U, int acc_S,
                            int n_cores, const int8_t* common, int64_t E, uint64_t seed, uint64_t off_offset,
                            uint64_t acc_offset, const uint64_t* offset_dev, int8_t* core_action, float* core_logprob,
                            int8_t* price_state, int8_t* price_action, float* price_logprob, int8_t* env_price,
                            int8_t* acc_action, float* acc_logprob, const float* ptab, const int16_t* pdigit,
                            int pkeys, int64_t pus, hipStream_t st) {
    if (!common || acc_stride < 16 || n_cores < 1 || acc_U % n_cores != 0) return hipErrorInvalidValue;
    ActArgs c = compact_args(acc, core_rows, core_owner, acc_stride, E, acc_U, acc_S, n_cores, common, seed,
                             acc_offset, offset_dev, nullptr, acc_action, acc_logprob);
    if (!price) {
        // a fixed-price round (cfg2): the offer units' one net (ActorCritic.act, k_act's single-net body) and the
        // compact acceptors in one launch
        ActArgs o{};
        o.n1 = *core;
        o.n2.n_groups = 0;
        o.obs = off_obs;
        o.stride = off_stride;
        o.U = off_U;
        o.S = off_S;
        o.E = (int)E;
        o.n_items = (int)(E * off_S);
        o.seed = seed;
        o.offset = off_offset;
        o.offset_dev = offset_dev;
        o.action = core_action;
        o.logprob = core_logprob;
        const bool paired = (off_stride + 31) / 32 == 1 && core->n_actions <= 16 && (acc_stride + 31) / 32 == 1 &&
                            acc->n_actions <= 16 && !env_int("MS_ACT_UNPAIRED", 0);
        if (paired && (!act_tiles_fits(o) || !act_common_fits(c))) return hipErrorInvalidValue;
        if (!paired) {
            hipError_t e = dispatch_act(o, st);
            return e != hipSuccess ? e : dispatch_act(c, st);
        }
        // wave split swept at cfg2 (profiles/r5g): 2048 offer / 512 acceptor target waves 8.5 us per launch (two
        // launches: 13.4 us; 1024 / 512: 8.8, 512 / 256: 9.4, 3072 / 512: 11.6, 2048 / 256: 10.8)
        static const long long f_off = env_int("MS_ACT_FIXED_WAVES", 2048), f_acc = env_int("MS_ACT_FIXED_COMMON_WAVES", 512);
        const unsigned ob = act_blocks(o, f_off), cb = act_common_blocks(c, f_acc);
        hipLaunchKernelGGL((k_act_pair<1, 1, 0, 1, 1>), dim3(ob + cb), dim3(256), 0, st, o, c, (int)ob);
        return hipGetLastError();
    }
    if (price->in_dim != 4) return hipErrorInvalidValue;
    ActArgs o = offer_free_args(core, price, off_obs, off_stride, E, off_U, off_S, n_cores, seed, off_offset,
                                offset_dev, nullptr, core_action, core_logprob, price_state, price_action,
                                price_logprob, env_price, pus);
    o.ptab = ptab;
    o.pdigit = pdigit;
    o.pkeys = pkeys;
    const bool unpaired = env_int("MS_ACT_UNPAIRED", 0) != 0;
    const bool paired = (off_stride + 31) / 32 == 1 && core->n_actions <= 16 && price->n_actions <= 16 &&
                        (acc_stride + 31) / 32 == 2 && acc->n_actions <= 32 && !unpaired;
    // cfg4's shapes (16 x 16 divided): 34-byte offer rows, 17 core actions, 99-byte acceptor rows, 49 actions
    const bool paired4 = !paired && (off_stride + 31) / 32 == 2 && core->n_actions <= 32 && price->n_actions <= 16 &&
                         (acc_stride + 31) / 32 == 4 && acc->n_actions <= 64 && !unpaired;
    if ((paired || paired4) && (!act_tiles_fits(o) || !act_common_fits(c))) return hipErrorInvalidValue;
    if (paired4) {
        // wave split swept at cfg4 (profiles/r6l, r6m): 1536 offer / 768 acceptor target waves 74.8 us per launch
        // (2048 / 1024: 80.3, 1024 / 1024: 78.4, 3072 / 1536: 78.2, 4096 / 1024: 84.3; two launches: 102.4)
        static const long long f4o = env_int("MS_ACT_PAIR4_WAVES", 1536), f4a = env_int("MS_ACT_PAIR4_COMMON_WAVES", 768);
        const unsigned ob = act_blocks(o, f4o), cb = act_common_blocks(c, f4a);
        hipLaunchKernelGGL((k_act_pair<2, 2, 1, 4, 4>), dim3(ob + cb), dim3(256), 0, st, o, c, (int)ob);
        return hipGetLastError();
    }
    if (!paired) {
        hipError_t e = dispatch_act(o, st);
        return e != hipSuccess ? e : dispatch_act(c, st);
    }
    // fewer, longer waves than either launch alone: the other half's waves fill the gaps
    // (the tools/gpu_job.sh waves step; profiles/r4af: 2048 / 768 -> 2048 offer and 2048 acceptor waves at cfg3)
    static const long long t_off = env_int("MS_ACT_PAIR_WAVES", 2048), t_acc = env_int("MS_ACT_PAIR_COMMON_WAVES", 768);
    const unsigned ob = act_blocks(o, t_off), cb = act_common_blocks(c, t_acc);
    hipLaunchKernelGGL((k_act_pair<1, 1, 1, 2, 2>), dim3(ob + cb), dim3(256), 0, st, o, c, (int)ob);
    return hipGetLastError();
}
#ifdef MS_ACT_PROBE_ON
// profiling build only: the paired act kernel's per-phase cycles, out[2][17] (the last column: waves)
extern "C" int ms_probe_act_cycles(unsigned long long* out, int clear) {
    static unsigned long long cyc[2][kActProbeWaves][16], waves[2][kActProbeWaves];
    if (hipMemcpyFromSymbol(cyc, HIP_SYMBOL(g_act_cycles), sizeof(cyc)) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(waves, HIP_SYMBOL(g_act_waves), sizeof(waves)) != hipSuccess) return -1;
    for (int h = 0; h < 2; h++) {
        for (int k = 0; k < 17; k++) out[17 * h + k] = 0;
        for (int w = 0; w < kActProbeWaves; w++) {
            for (int k = 0; k < 16; k++) out[17 * h + k] += cyc[h][w][k];
            out[17 * h + 16] += waves[h][w];
        }
    }
    if (clear) {
        memset(cyc, 0, sizeof(cyc));
        memset(waves, 0, sizeof(waves));
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_act_cycles), cyc, sizeof(cyc)) != hipSuccess) return -1;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_act_waves), waves, sizeof(waves)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
#endif

}  // namespace ms
