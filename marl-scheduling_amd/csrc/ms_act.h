// ms_act.h — the acting primitives shared by the act kernels (policy_kernels.hip) and the env round's
// fused acting of fixed-price global nets (env_kernels.hip): Philox2x32 uniforms, the exact three-term
// bf16 layer 1 (W1Split), the 16-wide head with its softmax / Categorical sampling (Head) and the act
// fragment block layout (ms_act_prepare). PPOmodules.py:53-63 (ActorCritic.act).
//
// Every includer gets the same floating-point contraction here (the policy kernels' -ffp-contract=fast),
// whatever its own flags, so the fused acting of the env kernel (built with contraction off) rounds
// exactly as k_act does. An includer restores its own setting after the include.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/marlsched.h"
#include "ms_common.h"

#pragma clang fp contract(fast)

namespace ms {

typedef float f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

__device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t& hi) {
    uint64_t p = (uint64_t)a * b;
    hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}

// Philox2x32-10 (Salmon et al., SC'11, the 2-word member of the family; BigCrush-clean from 7 rounds):
// two 32-bit outputs per (counter, key). The counter is (row, offset low word); the key folds in
// the 64-bit seed and the offset's high word. Half the multiplies of Philox4x32 for the two words
// a row needs (the act kernels' VALU budget: a 32-bit multiply issues at a quarter of the rate).
__device__ __forceinline__ void philox2(uint32_t row, uint64_t off, uint64_t seed, uint32_t& o0, uint32_t& o1) {
    uint32_t c0 = row, c1 = (uint32_t)off;
    uint32_t k = (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x85EBCA6Bu) ^ ((uint32_t)(off >> 32) * 0xC2B2AE35u);
#pragma unroll
    for (int r = 0; r < 10; r++) {
        uint32_t hi;
        const uint32_t lo = mulhilo(0xD256D193u, c0, hi);
        c0 = hi ^ k ^ c1;
        c1 = lo;
        k += 0x9E3779B9u;
    }
    o0 = c0;
    o1 = c1;
}

__device__ __forceinline__ float u24(uint32_t r) { return (float)(r >> 8) * (1.0f / 16777216.0f); }

__device__ __forceinline__ float xsum4g(float v) { return rows_sum(v); }

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma_bf16(const u4v& a, const u4v& b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                   0);
}

// tanh(x) = 1 - 2 / (1 + exp(2x)): exp overflows to inf for large x (-> 1) and underflows to 0 for
// large -x (-> -1); absolute error ~1e-7 (what feeds the next layers' sums of O(1) terms).
// tanh(a + b) with the bias pre-scaled, bs = b * 2 log2(e) (kTanhScale): the exponent is one fma
constexpr float kTanhScale = 2.8853900817779268f;
__device__ __forceinline__ float fast_tanh_b(float a, float bs) {
    const float t = __builtin_amdgcn_exp2f(fmaf(a, kTanhScale, bs));  // exp(2(a + b))
    return fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + t), 1.f);
}
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
// exp(x - m) as exp2(x log2e - m log2e) with one fma (m_l2e = m * log2e)
__device__ __forceinline__ float fast_exp_sub(float x, float m_l2e) {
    return __builtin_amdgcn_exp2f(fmaf(x, 1.4426950408889634f, -m_l2e));
}
__device__ __forceinline__ float fast_log(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }

// bf16 (upper half of the f32 bits) of elements 2i, 2i+1 packed into one dword
__device__ __forceinline__ uint32_t pack_hi(float lo, float hi) {
    return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);  // one v_perm_b32
}
__device__ __forceinline__ float trunc_bf16(float x) { return __uint_as_float(__float_as_uint(x) & 0xffff0000u); }

// Layer-1 weights as three bf16 terms, w = hi + mid + lo exactly (truncation leaves exact residuals),
// in the A-operand layout of v_mfma_f32_16x16x32_bf16 for k-step s: lane (i, g) holds
// W1[i][32s + 8g + 0..7].
template <int S1>
struct W1Split {
    u4v hi[S1], mid[S1], lo[S1];
    // the 12*S1 dwords of a lane's fragment (ms_act_prepare) in the act fragment block
    __device__ __forceinline__ void store_frag(uint32_t* f) const {
#pragma unroll
        for (int s = 0; s < S1; s++) {
            *reinterpret_cast<u4v*>(f + 12 * s) = hi[s];
            *reinterpret_cast<u4v*>(f + 12 * s + 4) = mid[s];
            *reinterpret_cast<u4v*>(f + 12 * s + 8) = lo[s];
        }
    }
    __device__ __forceinline__ void load_frag(const uint32_t* f) {
#pragma unroll
        for (int s = 0; s < S1; s++) {
            hi[s] = *reinterpret_cast<const u4v*>(f + 12 * s);
            mid[s] = *reinterpret_cast<const u4v*>(f + 12 * s + 4);
            lo[s] = *reinterpret_cast<const u4v*>(f + 12 * s + 8);
        }
    }
    __device__ void load(const float* w1 /* [16][D] of this group */, int D, int i, int g) {
#pragma unroll
        for (int s = 0; s < S1; s++) {
            float h[8], m[8], l[8];
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const int k = 32 * s + 8 * g + e;
                const float w = k < D ? w1[i * D + k] : 0.f;
                h[e] = trunc_bf16(w);
                const float r1 = w - h[e];
                m[e] = trunc_bf16(r1);
                l[e] = r1 - m[e];  // <= 8 significant bits: exact in bf16
            }
#pragma unroll
            for (int d = 0; d < 4; d++) {
                hi[s][d] = pack_hi(h[2 * d], h[2 * d + 1]);
                mid[s][d] = pack_hi(m[2 * d], m[2 * d + 1]);
                lo[s][d] = pack_hi(l[2 * d], l[2 * d + 1]);
            }
        }
    }
};

// int8 observation bytes (two dwords = 8 consecutive inputs) as a bf16 B fragment (exact)
__device__ __forceinline__ u4v bytes_to_bf16(uint32_t d0, uint32_t d1) {
    u4v r;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const uint32_t src = d < 2 ? d0 : d1;
        const int sh = 16 * (d & 1);
        const float a = (float)(int8_t)(src >> sh);
        const float b = (float)(int8_t)(src >> (sh + 8));
        r[d] = pack_hi(a, b);
    }
    return r;
}

// The 16-wide layers and the head of one net, in registers: lane (j, g4) holds W2[j][4*g4 + s],
// W3[16t + j][4*g4 + s] (the permuted-k A operands) and the biases of its accumulator rows.
template <int NT>
struct Head {
    float b1[4], w2[4], b2[4], w3[NT][4], b3[NT][4];  // b1, b2 pre-scaled by kTanhScale (fast_tanh_b)
    static constexpr int FW = 12 + 8 * NT;  // dwords of a lane's fragment
    __device__ __forceinline__ void store_frag(float* f) const {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            f[q] = b1[q];
            f[4 + q] = w2[q];
            f[8 + q] = b2[q];
#pragma unroll
            for (int t = 0; t < NT; t++) {
                f[12 + 4 * t + q] = w3[t][q];
                f[12 + 4 * NT + 4 * t + q] = b3[t][q];
            }
        }
    }
    __device__ __forceinline__ void load_frag(const float* f) {
#pragma unroll
        for (int q4 = 0; q4 < 3 + 2 * NT; q4++) {
            const f4 v = *reinterpret_cast<const f4*>(f + 4 * q4);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float x = v[q];
                if (q4 == 0) b1[q] = x;
                else if (q4 == 1) w2[q] = x;
                else if (q4 == 2) b2[q] = x;
                else if (q4 < 3 + NT) w3[q4 - 3][q] = x;
                else b3[q4 - 3 - NT][q] = x;
            }
        }
    }
    __device__ void load(const ms_mlp_params& p, int grp, int j, int g4) {
        const int A = p.n_actions;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            b1[q] = p.b1[grp * 16 + 4 * g4 + q] * kTanhScale;
            w2[q] = p.w2[(size_t)grp * 256 + j * 16 + 4 * g4 + q];
            b2[q] = p.b2[grp * 16 + 4 * g4 + q] * kTanhScale;
#pragma unroll
            for (int t = 0; t < NT; t++) {
                const int a = 16 * t + j, ab = 16 * t + 4 * g4 + q;
                w3[t][q] = a < A ? p.w3[((size_t)grp * A + a) * 16 + 4 * g4 + q] : 0.f;
                b3[t][q] = ab < A ? p.b3[(size_t)grp * A + ab] : -INFINITY;  // padding actions: exp -> 0
            }
        }
    }

    // Layers 2-3 and the softmax numerators of the 16 rows of a tile given layer-1 pre-activations:
    // z[t][q] = exp(logit - max) of action a = 16t + 4*g4 + q of row j, S = the row's sum of z and
    // c[t][q] = the running sum of z over actions 0..a (in increasing action order). Logits of the
    // padding actions (a >= A) read -inf (bias), so they drop out of the max and the sums.
    __device__ __forceinline__ void numerators(f4 a1, int j, int g4, float (&z)[NT][4], float (&c)[NT][4],
                                               float& S) const {
        float h1[4];
#pragma unroll
        for (int q = 0; q < 4; q++) h1[q] = fast_tanh_b(a1[q], b1[q]);
        f4 a2 = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 4; s++) a2 = mfma4(w2[s], h1[s], a2);
        float h2[4];
#pragma unroll
        for (int q = 0; q < 4; q++) h2[q] = fast_tanh_b(a2[q], b2[q]);
        float m = -INFINITY;
#pragma unroll
        for (int t = 0; t < NT; t++) {
            f4 zz = {0, 0, 0, 0};
#pragma unroll
            for (int s = 0; s < 4; s++) zz = mfma4(w3[t][s], h2[s], zz);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                z[t][q] = zz[q] + b3[t][q];
                m = fmaxf(m, z[t][q]);
            }
        }
        m = rows_max(m);
        float bs[NT];
        const float m_l2e = m * 1.4426950408889634f;
#pragma unroll
        for (int t = 0; t < NT; t++) {
            bs[t] = 0.f;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                z[t][q] = fast_exp_sub(z[t][q], m_l2e);
                bs[t] += z[t][q];
            }
        }
        float lane_tot = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++) lane_tot += bs[t];
        // (one 16-action tile: S is the running sums' total, (gs0 + gs1) + (gs2 + gs3), which is
        //  xsum4g(lane_tot) bit for bit)
        if (NT > 1) S = xsum4g(lane_tot);
        float cum = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++) {
            uint32_t gsr[4];
            rows_bcast(__float_as_uint(bs[t]), gsr);
            const float gs0 = __uint_as_float(gsr[0]), gs1 = __uint_as_float(gsr[1]), gs2 = __uint_as_float(gsr[2]),
                        gs3 = __uint_as_float(gsr[3]);
            float cc = cum + (g4 > 0 ? gs0 : 0.f) + (g4 > 1 ? gs1 : 0.f) + (g4 > 2 ? gs2 : 0.f);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                cc += z[t][q];
                c[t][q] = cc;
            }
            cum += (gs0 + gs1) + (gs2 + gs3);
        }
        if (NT == 1) S = cum;
    }

    // run() of two tiles side by side: their MFMA chains and transcendentals interleave, and their
    // cross-lane reductions pair up (rows_max2, rows_sum2, rows_sum2_i). The running sums are compared
    // with u * S as they are formed instead of being kept. Bit-identical to two run() calls.
    __device__ __forceinline__ void run2(const f4 (&a1)[2], int A, int g4, const float (&u)[2], int (&action)[2],
                                         float (&logprob)[2]) const {
        float h1[2][4];
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) h1[i][q] = fast_tanh_b(a1[i][q], b1[q]);
        f4 a2[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
            for (int i = 0; i < 2; i++) a2[i] = mfma4(w2[s], h1[i][s], a2[i]);
        float h2[2][4];
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) h2[i][q] = fast_tanh_b(a2[i][q], b2[q]);
        float z[2][NT][4];
        float m[2] = {-INFINITY, -INFINITY};
#pragma unroll
        for (int t = 0; t < NT; t++) {
            f4 zz[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int i = 0; i < 2; i++) zz[i] = mfma4(w3[t][s], h2[i][s], zz[i]);
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    z[i][t][q] = zz[i][q] + b3[t][q];
                    m[i] = fmaxf(m[i], z[i][t][q]);
                }
        }
        rows_max2(m[0], m[1]);
        float bs[2][NT], S[2];
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const float m_l2e = m[i] * 1.4426950408889634f;
            S[i] = 0.f;
#pragma unroll
            for (int t = 0; t < NT; t++) {
                bs[i][t] = 0.f;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    z[i][t][q] = fast_exp_sub(z[i][t][q], m_l2e);
                    bs[i][t] += z[i][t][q];
                }
            }
#pragma unroll
            for (int t = 0; t < NT; t++) S[i] += bs[i][t];
        }
        int cnt[2];
        if (NT > 1) {
            rows_sum2(S[0], S[1]);  // = xsum4g(lane_tot) of numerators()
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const float target = u[i] * S[i];
                float cum = 0.f;
                cnt[i] = 0;
#pragma unroll
                for (int t = 0; t < NT; t++) {
                    uint32_t gsr[4];
                    rows_bcast(__float_as_uint(bs[i][t]), gsr);
                    const float gs0 = __uint_as_float(gsr[0]), gs1 = __uint_as_float(gsr[1]),
                                gs2 = __uint_as_float(gsr[2]), gs3 = __uint_as_float(gsr[3]);
                    float cc = cum + (g4 > 0 ? gs0 : 0.f) + (g4 > 1 ? gs1 : 0.f) + (g4 > 2 ? gs2 : 0.f);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        cc += z[i][t][q];
                        cnt[i] += (cc <= target) ? 1 : 0;
                    }
                    cum += (gs0 + gs1) + (gs2 + gs3);
                }
            }
        } else {
            // one 16-action tile: S is the running sums' total (gs0 + gs1) + (gs2 + gs3), known only
            // after the broadcast, so the running sums are kept for the compare
            float c[2][4];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                uint32_t gsr[4];
                rows_bcast(__float_as_uint(bs[i][0]), gsr);
                const float gs0 = __uint_as_float(gsr[0]), gs1 = __uint_as_float(gsr[1]), gs2 = __uint_as_float(gsr[2]),
                            gs3 = __uint_as_float(gsr[3]);
                const float cum = 0.f;  // numerators()' expression, term for term
                float cc = cum + (g4 > 0 ? gs0 : 0.f) + (g4 > 1 ? gs1 : 0.f) + (g4 > 2 ? gs2 : 0.f);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    cc += z[i][0][q];
                    c[i][q] = cc;
                }
                S[i] = cum + ((gs0 + gs1) + (gs2 + gs3));
                const float target = u[i] * S[i];
                cnt[i] = 0;
#pragma unroll
                for (int q = 0; q < 4; q++) cnt[i] += (c[i][q] <= target) ? 1 : 0;
            }
        }
        rows_sum2_i(cnt[0], cnt[1]);
        if (__builtin_expect(__ballot(cnt[0] >= A || cnt[1] >= A) != 0, 0)) {
            // u * S at or beyond the rounded total: the last action with nonzero probability
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int last_nz = last_nonzero(z[i], g4);
                if (cnt[i] >= A) cnt[i] = last_nz;
            }
        }
        float mine[2] = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int q = 0; q < 4; q++) mine[i] = (16 * t + 4 * g4 + q == cnt[i]) ? z[i][t][q] : mine[i];
        rows_sum2(mine[0], mine[1]);
#pragma unroll
        for (int i = 0; i < 2; i++) {
            action[i] = cnt[i];
            logprob[i] = clamped_log(mine[i] * __builtin_amdgcn_rcpf(S[i]));
        }
    }

    __device__ __forceinline__ static int last_nonzero(const float (&z)[NT][4], int g4) {
        int last_nz = -1;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (z[t][q] > 0.f) last_nz = 16 * t + 4 * g4 + q;
        last_nz = rows_max_i(last_nz);
        return last_nz;
    }

    __device__ __forceinline__ static float clamped_log(float pa) {
        const float eps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps
        return fast_log(fminf(fmaxf(pa, eps), 1.f - eps));
    }

    // The sampling entries of the tile's 16 rows, one row per column j: lane (j, g4) gets its four
    // actions' running sums c and log-probs lp (what run() would compare and return), and S and the
    // last nonzero action of row j (every lane of the row).
    __device__ __forceinline__ void row_table(f4 a1, int j, int g4, float (&c)[NT][4], float (&lp)[NT][4], float& S,
                                              int& last_nz) const {
        float z[NT][4];
        numerators(a1, j, g4, z, c, S);
        last_nz = last_nonzero(z, g4);
        const float rS = __builtin_amdgcn_rcpf(S);
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) lp[t][q] = clamped_log(z[t][q] * rS);
    }

    // The sampling table of one row (all 16 rows of the tile equal): cum[a] = running sum through
    // action a, lp[a] = the log-prob run() returns for action a, *S and *last_nz. With it, a row equal
    // to this one samples and scores exactly as run() would.
    __device__ __forceinline__ void table(f4 a1, int j, int g4, float* cum, float* lp, float* S_out,
                                          int* last_nz_out) const {
        float z[NT][4], c[NT][4], S;
        numerators(a1, j, g4, z, c, S);
        const int last_nz = last_nonzero(z, g4);
        if (j == 0) {
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int a = 16 * t + 4 * g4 + q;
                    cum[a] = c[t][q];
                    lp[a] = clamped_log(z[t][q] * __builtin_amdgcn_rcpf(S));
                }
            if (g4 == 0) {
                *S_out = S;
                *last_nz_out = last_nz;
            }
        }
    }
};

// ---- act fragment block (ms_act_prepare): a header {magic, S1, NT, has common table}, then per group
//      [64 lanes][LW] dwords (the lane's W1Split<S1> terms and Head<NT> parameters, exactly what the
//      acting wave would derive) and the common row's sampling table [16 NT running sums][16 NT
//      log-probs][S][last nonzero][2 pad] (Head::table)
constexpr uint32_t kFragMagic = 0x4D534641u;
template <int S1, int NT>
struct FragLayout {
    static constexpr int LW = 12 * S1 + Head<NT>::FW;  // dwords per lane (a multiple of 4)
    static constexpr int TB = 32 * NT + 4;              // common table dwords
    static constexpr int GB = 64 * LW + TB;             // dwords per group
};
// the group blocks of p's fragment block, or NULL when it is absent or made for another shape
template <int S1, int NT>
__device__ __forceinline__ const uint32_t* frag_groups(const ms_mlp_params& p, bool need_common) {
    const uint32_t* f = static_cast<const uint32_t*>(p.act_frag);
    if (!f) return nullptr;
    const uint32_t h0 = __builtin_amdgcn_readfirstlane(f[0]), h1 = __builtin_amdgcn_readfirstlane(f[1]),
                   h2 = __builtin_amdgcn_readfirstlane(f[2]), h3 = __builtin_amdgcn_readfirstlane(f[3]);
    if (h0 != kFragMagic || h1 != (uint32_t)S1 || h2 != (uint32_t)NT || (need_common && !h3)) return nullptr;
    return f + 4;
}

// The common row's sampling table (Head::table) into LDS: its dwords (zero past the row: they meet
// zero weights, like k_act's clamped loads) through layer 1 and the head. One wave.
template <int S1, int NT>
__device__ __forceinline__ void common_table(const W1Split<S1>& w1, const Head<NT>& h1, const int8_t* common,
                                             int stride4, uint32_t* tmpl, float* cum, float* lp, float* S, int* lnz,
                                             int lane) {
    const int j = lane & 15, g4 = lane >> 4;
    const uint32_t* crow = reinterpret_cast<const uint32_t*>(common);
    for (int d = lane; d < 8 * S1; d += 64) tmpl[d] = d < stride4 ? crow[d] : 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < S1; s++) {
        const u4v x = bytes_to_bf16(tmpl[8 * s + 2 * g4], tmpl[8 * s + 2 * g4 + 1]);
        acc = mfma_bf16(w1.hi[s], x, acc);
        acc = mfma_bf16(w1.mid[s], x, acc);
        acc = mfma_bf16(w1.lo[s], x, acc);
    }
    h1.table(acc, j, g4, cum, lp, S, lnz);
}

}  // namespace ms
