// bdqn_kernels.hip — Branching DQN acting (BranchingDQNModules.py:75-123) for BASELINE cfg5 on gfx950.
//
// BranchingQNetwork: out = ReLU(W2 ReLU(W1 x + b1) + b2), value = wv out + bv, per branch b
// adv_b = Wa_b out + ba_b, q_b = value + adv_b - mean(adv_b) (:88-101); get_action takes the
// argmax of every branch (torch.argmax: the first maximum, :117-123). At cfg5 every frame acts
// for E * N = 262144 agents: the acceptor role's heads alone are [262144, 128] x [128, 32 * 97],
// 208 GFLOP, and a library GEMM materialises 3.25 GB of advantages that an argmax pass reads
// back. Here:
//
//   k_bdqn_w1split    W1 as three bf16 terms (hi + mid + lo = W1 exactly), zero-padded per input
//                     segment, once per weight update;
//   k_bdqn_l1_cf /    W1_c F per core c (F = the foreign acceptor row, Agent.py:167-212) and
//   k_bdqn_l1_base    base = b1 + sum_c W1_c F, once per weight update;
//   k_bdqn_l1_cores   layer 1 of all N agents' aggregated acceptor rows from the compact
//   k_bdqn_l1_gather  observations: an agent's row is R_c on the cores it owns and F elsewhere, so
//                     W1 x_a + b1 = base + sum_{c owned by a} P_c, P_c = W1_c R_c - W1_c F of every
//                     (replica, core) on v_mfma_f32_16x16x32_bf16 (the int8 row bytes are exact in
//                     bf16 and W1 is three exact bf16 terms: exact products, f32 accumulation); the
//                     gather adds an agent's owned cores' P rows to base in core order (the h1 rows of
//                     ms_bdqn_layer1_compact; ms_bdqn_act_compact does that sum inside k_bdqn_act);
//   k_bdqn_own_mask / the compact acting's row list: only agents that own a core run the heads, the
//   k_bdqn_own_list / others (layer 1 = base) take the one common row's greedy actions (fill);
//   k_bdqn_common_fill
//   k_bdqn_act        the trunk, the value head and every advantage head fused with the per-branch
//                     mean, q and first-maximum argmax, then the epsilon-greedy pick: nothing but
//                     the int8 actions leaves the kernel. Trunk and heads run on
//                     v_mfma_f32_16x16x32_bf16 with both operands as three exact bf16 terms and six
//                     products (the f32 product sum within about f32 rounding, see the comment at the
//                     kernel). The batch is on the MFMA column axis and every layer's accumulator is
//                     the next layer's B operand (the K order permuted to match); a block of 8 waves
//                     (256 rows, two 16-row tiles per wave) stages W2's terms, then one branch's Wa
//                     rows at a time in LDS (the next branch's f32 rows arrive by LDS-DMA during the
//                     current one's MFMAs). With h1 == NULL and P == NULL layer 1 runs in the kernel
//                     on int8 rows (the offerer / price roles).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/marlsched.h"
#include "ms_bdqn.h"
#include "ms_common.h"

namespace ms {

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 mfma_bf16(const u4v& a, const u4v& b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                   0);
}
__device__ __forceinline__ uint32_t pack_hi(float lo, float hi) {
    return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);
}
__device__ __forceinline__ uint32_t pack_i(int a, int b) { return pack_hi((float)a, (float)b); }
__device__ __forceinline__ float trunc_bf16(float x) { return __uint_as_float(__float_as_uint(x) & 0xffff0000u); }

// eight f32 values as three exact bf16 terms (hi + mid + lo == v: each term keeps 8 significant bits)
__device__ __forceinline__ void split8(const float (&v)[8], u4v& hi, u4v& mid, u4v& lo) {
#pragma unroll
    for (int t = 0; t < 4; t++) {
        float h[2], m[2], l[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const float x = v[2 * t + u];
            h[u] = trunc_bf16(x);
            const float r = x - h[u];
            m[u] = trunc_bf16(r);
            l[u] = r - m[u];
        }
        hi[t] = pack_hi(h[0], h[1]);
        mid[t] = pack_hi(m[0], m[1]);
        lo[t] = pack_hi(l[0], l[1]);
    }
}

// the foreign acceptor row F (Agent.py:167-212): [0, -1, -1, (-2, -2) * O]; zero past D
__device__ __forceinline__ int foreign(int k, int D) { return k == 0 ? 0 : (k <= 2 ? -1 : (k < D ? -2 : 0)); }

}  // namespace

// ---- W1 [128][segs * seg] -> three bf16 terms [3][128][segs][Dp] (zero for k >= seg)
__global__ void __launch_bounds__(256) k_bdqn_w1split(const float* __restrict__ w1, int seg, int segs, int Dp,
                                                      uint16_t* __restrict__ out) {
    const long long total = (long long)kBH * segs * Dp;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
        const int k = (int)(i % Dp);
        const long long hs = i / Dp;  // h * segs + sg
        const int sg = (int)(hs % segs), h = (int)(hs / segs);
        const float w = k < seg ? w1[(size_t)h * segs * seg + (size_t)sg * seg + k] : 0.f;
        const float hi = trunc_bf16(w), r = w - hi, mid = trunc_bf16(r), lo = r - mid;
        out[i] = (uint16_t)(__float_as_uint(hi) >> 16);
        out[total + i] = (uint16_t)(__float_as_uint(mid) >> 16);
        out[2 * total + i] = (uint16_t)(__float_as_uint(lo) >> 16);
    }
}

// ---- cF[c][h] = sum_k W1[h][c*D + k] F[k] (block (h, c), a fixed-order tree over its 256 threads), then
//      base[h] = b1[h] + sum_c cF[c][h] in core order
__global__ void __launch_bounds__(256) k_bdqn_l1_cf(const float* __restrict__ w1, int D, int C, float* __restrict__ cF) {
    __shared__ float red[256];
    const int h = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
    float s = 0.f;
    for (int k = t; k < D; k += 256) s = fmaf(w1[(size_t)h * C * D + (size_t)c * D + k], (float)foreign(k, D), s);
    red[t] = s;
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
        if (t < d) red[t] += red[t + d];
        __syncthreads();
    }
    if (t == 0) cF[(size_t)c * kBH + h] = red[0];
}
__global__ void __launch_bounds__(128) k_bdqn_l1_base(const float* __restrict__ cF, const float* __restrict__ b1, int C,
                                                      float* __restrict__ base) {
    const int h = threadIdx.x;
    float s = 0.f;
    for (int c = 0; c < C; c++) s += cF[(size_t)c * kBH + h];
    base[h] = b1[h] + s;
}

// ---- layer 1 from compact observations, two passes.
//      k_bdqn_l1_cores: P[e][c] = W1_c R_ec - W1_c F for every (replica, core): the accumulator starts
//      at -cF[c] (ms_bdqn_prepare) and the int8 row bytes go to the bf16 B operand as they are (exact;
//      the split W1 is zero past D, so the row's padding bytes add nothing). A wave owns one (core,
//      16 hidden) tile and holds its A fragments (three bf16 terms of every k-step) in registers
//      while it walks replica tiles of 16: only the int8 rows stream in and P streams out.
//      k_bdqn_l1_gather: h1[e*N + a] = base + the P rows of the cores agent a owns, in core order (an
//      agent owns at most L cores: its free slots bound them, world.py:369-376).
constexpr int kL1MaxSteps = 8;  // k-steps of 32 inputs per core (D <= 256)
constexpr int kL1TilesPerWave = 8;

template <int S>
__global__ void __launch_bounds__(256) k_bdqn_l1_cores(BdqnL1Compact p) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int i = lane & 15, g4 = lane >> 4;
    const long long gw = (long long)blockIdx.x * 4 + (tid >> 6);
    const int C = p.C, Dp = p.Dp;
    const long long rtiles = (p.E + 15) / 16;
    const long long chunks = (rtiles + kL1TilesPerWave - 1) / kL1TilesPerWave;
    // wave -> (core, hidden tile, replica chunk); the 8 hidden tiles of a (core, chunk) are neighbours
    const int ht = (int)(gw & 7);
    const long long rest = gw >> 3;
    const int c = (int)(rest % C);
    const long long ch = rest / C;
    if (ch >= chunks) return;
    const int stride4 = p.stride >> 2;
    const size_t tsz = (size_t)kBH * C * Dp;
    const uint16_t* wp0 = p.w1s + ((size_t)(16 * ht + i) * C + c) * Dp + 8 * g4;
    u4v aw[S][3];
#pragma unroll
    for (int s = 0; s < S; s++)
#pragma unroll
        for (int t = 0; t < 3; t++) aw[s][t] = *reinterpret_cast<const u4v*>(wp0 + t * tsz + 32 * s);
    const long long t0 = ch * kL1TilesPerWave, t1 = min(t0 + kL1TilesPerWave, rtiles);
    // register prefetch: the next replica tile's row dwords are loaded before this tile's MFMAs
    auto load_tile = [&](long long rt, uint32_t (&xw)[S][2]) {
        const long long e = rt * 16 + i;
        const uint32_t* row = reinterpret_cast<const uint32_t*>(p.core_rows + ((size_t)(e < p.E ? e : 0) * C + c) * p.stride);
#pragma unroll
        for (int s = 0; s < S; s++) {
            const int d0 = 8 * s + 2 * g4;
            xw[s][0] = d0 < stride4 ? row[d0] : 0u;
            xw[s][1] = d0 + 1 < stride4 ? row[d0 + 1] : 0u;
        }
    };
    const f4 ncf = -*reinterpret_cast<const f4*>(p.cF + (size_t)c * kBH + 16 * ht + 4 * g4);
    // two replica tiles per step, one accumulator per (tile, W1 term): six independent MFMA chains, and the
    // next pair's rows in flight during this pair's MFMAs
    uint32_t cur[2][S][2];
    load_tile(t0, cur[0]);
    load_tile(t0 + 1 < t1 ? t0 + 1 : t0, cur[1]);
    for (long long rt = t0; rt < t1; rt += 2) {
        uint32_t nxt[2][S][2];
        if (rt + 2 < t1) {
            load_tile(rt + 2, nxt[0]);
            load_tile(rt + 3 < t1 ? rt + 3 : rt + 2, nxt[1]);
        }
        f4 acc[2][3];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            acc[u][0] = ncf;
            acc[u][1] = acc[u][2] = (f4){0, 0, 0, 0};
        }
#pragma unroll
        for (int s = 0; s < S; s++) {
            u4v xb[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                xb[u][0] = pack_i((int8_t)cur[u][s][0], (int8_t)(cur[u][s][0] >> 8));
                xb[u][1] = pack_i((int8_t)(cur[u][s][0] >> 16), (int8_t)(cur[u][s][0] >> 24));
                xb[u][2] = pack_i((int8_t)cur[u][s][1], (int8_t)(cur[u][s][1] >> 8));
                xb[u][3] = pack_i((int8_t)(cur[u][s][1] >> 16), (int8_t)(cur[u][s][1] >> 24));
            }
#pragma unroll
            for (int t = 0; t < 3; t++)
#pragma unroll
                for (int u = 0; u < 2; u++) acc[u][t] = mfma_bf16(aw[s][t], xb[u], acc[u][t]);
        }
        // lane (replica i, g4) holds P_c[hidden 16 ht + 4 g4 + q] of replica e
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const long long e = (rt + u) * 16 + i;
            if (rt + u < t1 && e < p.E)
                *reinterpret_cast<f4*>(p.P + ((size_t)e * C + c) * kBH + 16 * ht + 4 * g4) =
                    (acc[u][0] + acc[u][1]) + acc[u][2];
        }
        if (rt + 2 < t1) {
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
                for (int s2 = 0; s2 < S; s2++) cur[u][s2][0] = nxt[u][s2][0], cur[u][s2][1] = nxt[u][s2][1];
        }
    }
}

// thread = one float4 of one agent row: base + its owned cores' P rows in core order
__global__ void __launch_bounds__(256) k_bdqn_l1_gather(BdqnL1Compact p) {
    const long long x = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long rows = p.E * p.N;
    if (x >= rows * 32) return;
    const long long r = x >> 5;
    const int h4 = (int)(x & 31);
    const long long e = r / p.N;
    const int a1 = (int)(r - e * p.N) + 1;
    const int8_t* own = p.core_owner + (size_t)e * p.C;
    f4 v = *reinterpret_cast<const f4*>(p.base + 4 * h4);
    for (int c = 0; c < p.C; c++)
        if (own[c] == a1) v += *reinterpret_cast<const f4*>(p.P + ((size_t)e * p.C + c) * kBH + 4 * h4);
    *reinterpret_cast<f4*>(p.h1 + (size_t)r * kBH + 4 * h4) = v;
}

// ---- the rows of agents that own a core (the others' acceptor row is the common row F everywhere, so
//      their layer 1 is base and their greedy actions are the common row's). k_bdqn_own_mask: per replica
//      the bitmask of agents owning a core (N <= 64); k_bdqn_own_list: one atomic per wave (ballot +
//      prefix count) appends the owning rows; the list order varies from run to run, each row's result
//      does not. Entry 0 is the common row itself (-1).
__global__ void __launch_bounds__(256) k_bdqn_own_mask(BdqnAct p, unsigned long long* mask) {
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    // k_bdqn_own_list's counter starts at zero (here, not a hipMemsetAsync: see k_key_clear)
    if (e == 0) *const_cast<int32_t*>(p.n_owning) = 0;
    if (e >= p.rows / p.N) return;
    const int8_t* own = p.core_owner + (size_t)e * p.C;
    unsigned long long m = 0;
    if ((p.C & 15) == 0) {
        for (int c = 0; c < p.C; c += 16) {
            const uint4 v = *reinterpret_cast<const uint4*>(own + c);
            const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int o = (int)(int8_t)(d[k >> 2] >> (8 * (k & 3)));
                if (o > 0) m |= 1ull << (o - 1);
            }
        }
    } else {
        for (int c = 0; c < p.C; c++) {
            const int o = own[c];
            if (o > 0) m |= 1ull << (o - 1);
        }
    }
    mask[e] = m;
}
constexpr int kOwnListThreads = 1024;  // rows per block of k_bdqn_own_list: one atomic per block
__global__ void __launch_bounds__(kOwnListThreads) k_bdqn_own_list(BdqnAct p, const unsigned long long* mask,
                                                                   int32_t* list, int32_t* count) {
    __shared__ int wcount[kOwnListThreads / 64];
    __shared__ int bbase;
    const long long r = (long long)blockIdx.x * kOwnListThreads + threadIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    bool owns = false;
    if (r < p.rows) {
        const long long e = r / p.N;
        owns = (mask[e] >> (int)(r - e * p.N)) & 1ull;
    }
    const unsigned long long m = __ballot(owns);
    if (lane == 0) wcount[w] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int k = 0; k < kOwnListThreads / 64; k++) {
            const int c = wcount[k];
            wcount[k] = tot;  // exclusive offsets of the waves
            tot += c;
        }
        bbase = tot ? atomicAdd(count, tot) : 0;
    }
    __syncthreads();
    if (owns) list[1 + bbase + wcount[w] + __popcll(m & ((1ull << lane) - 1))] = (int32_t)r;
    if (r == 0) list[0] = -1;
}

// ---- rows of agents owning no core: the common row's greedy actions (or the row's random ones)
__global__ void __launch_bounds__(256) k_bdqn_common_fill(BdqnAct p, const unsigned long long* mask) {
    const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
    if (r >= p.rows) return;
    const long long e = r / p.N;
    if ((mask[e] >> (int)(r - e * p.N)) & 1ull) return;
    const int A = p.q.ac_dim;
    const int8_t* src = (p.explore && p.explore[r] != 0) ? p.rnd + (size_t)r * A : p.common;
    int8_t* dst = p.action + (size_t)r * A;
    if ((A & 15) == 0) {
        for (int b = 0; b < A; b += 16) *reinterpret_cast<uint4*>(dst + b) = *reinterpret_cast<const uint4*>(src + b);
    } else {
        for (int b = 0; b < A; b++) dst[b] = src[b];
    }
}

// ---- the fused trunk + heads + argmax. Block = 8 waves x 32 rows: two 16-row column tiles per wave;
//      lane (j, g4): row j of each of its wave's tiles, k-group / accumulator-row group g4.
//      Heads on v_mfma_f32_16x16x32_bf16 with both operands as three exact bf16 terms (W = a1 + a2 + a3,
//      out = b1 + b2 + b3, each term 8 significant bits): the six products down to 2^-16 of the leading
//      one (a1 b1; a1 b2, a2 b1; a1 b3, a2 b2, a3 b1) are exact in the f32 accumulator, the three
//      dropped ones are below 2^-23 of it, so a q value differs from the f32 product sum by about f32
//      rounding (3 MFMA passes of 16 cycles per 32 inputs instead of 8 of 32 on v_mfma_f32_16x16x4_f32).
//      K permutation of the heads: k-step s, lane group g4, element e <-> hidden unit
//      16 (2 s + e / 4) + 4 g4 + e % 4, so a lane's B fragment is its own trunk outputs out[2s], out[2s+1]
//      and the staged Wa rows are stored permuted to match.
constexpr int kAPitch = 136;    // bf16 pitch of a staged term row (272 B: 16 rows' b128 reads spread over the banks)
// hidden units 4 k4 .. 4 k4 + 3 (= 16 kt + 4 g + 0..3) of a 128-wide weight row m as three bf16 terms,
// stored at positions 32 (kt / 2) + 8 g + 4 (kt % 2) + 0..3 of term rows [3][rows][kAPitch]: the
// permuted K order whose k-step s, lane group g4, element e is hidden unit 16 (2 s + e / 4) + 4 g4 + e % 4
__device__ __forceinline__ void put_terms(uint16_t* base, int rows, int m, int k4, const f4& v4) {
    const int kt = k4 >> 2, g = k4 & 3;
    const int pos = 32 * (kt >> 1) + 8 * g + 4 * (kt & 1);
    uint32_t t3[3][2];
#pragma unroll
    for (int e2 = 0; e2 < 2; e2++) {
        float hh[2], mm[2], ll[2];
#pragma unroll
        for (int u2 = 0; u2 < 2; u2++) {
            const float v = v4[2 * e2 + u2];
            hh[u2] = trunc_bf16(v);
            const float r = v - hh[u2];
            mm[u2] = trunc_bf16(r);
            ll[u2] = r - mm[u2];
        }
        t3[0][e2] = pack_hi(hh[0], hh[1]);
        t3[1][e2] = pack_hi(mm[0], mm[1]);
        t3[2][e2] = pack_hi(ll[0], ll[1]);
    }
#pragma unroll
    for (int t = 0; t < 3; t++)
        *reinterpret_cast<uint2*>(base + ((size_t)t * rows + m) * kAPitch + pos) = make_uint2(t3[t][0], t3[t][1]);
}
// six products of the three-term operands into one accumulator (the three below 2^-23 of the leading
// product dropped)
__device__ __forceinline__ f4 mfma_split6(const u4v& a1, const u4v& a2, const u4v& a3, const u4v (&b)[3], f4 c) {
    c = mfma_bf16(a1, b[0], c);
    c = mfma_bf16(a1, b[1], c);
    c = mfma_bf16(a2, b[0], c);
    c = mfma_bf16(a1, b[2], c);
    c = mfma_bf16(a2, b[1], c);
    c = mfma_bf16(a3, b[0], c);
    return c;
}

constexpr int kActWaves = 8;
constexpr int kActTiles = 2;    // 16-row column tiles per wave

template <int NMT, bool L1>
__global__ void __launch_bounds__(64 * kActWaves) k_bdqn_act(BdqnAct p) {
    constexpr int ROWS_W = 16 * NMT;                   // staged Wa rows per branch
    constexpr int NTH = 64 * kActWaves;
    constexpr int NC = kActTiles;
    extern __shared__ __align__(16) float sm[];        // [128][kBPitch] W2, then [3][ROWS_W][kAPitch] bf16 Wa + ba
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int j = lane & 15, g4 = lane >> 4;
    const int n = p.q.n, A = p.q.ac_dim;
    const long long row0 = ((long long)blockIdx.x * kActWaves + w) * 16 * NC;
    long long row[NC], rc[NC];
    bool rv[NC], virt[NC];
    if (p.list) {
        // row list: positions past 1 + *n_owning exit (the whole block: before any barrier)
        const long long nl = 1 + (long long)__builtin_amdgcn_readfirstlane(*p.n_owning);
        if ((long long)blockIdx.x * kActWaves * 16 * NC >= nl) return;
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const long long lp = row0 + 16 * c + j;
            const int r = p.list[lp < nl ? lp : nl - 1];
            virt[c] = lp < nl && r < 0;
            rv[c] = lp < nl && r >= 0;
            row[c] = r < 0 ? 0 : r;
            rc[c] = row[c];
        }
    } else {
#pragma unroll
        for (int c = 0; c < NC; c++) {
            row[c] = row0 + 16 * c + j;
            rv[c] = row[c] < p.rows;
            virt[c] = false;
            rc[c] = rv[c] ? row[c] : p.rows - 1;
        }
    }

    // stage W2 as three bf16 terms in the permuted K order ([3][128][kAPitch])
    uint16_t* sW2 = reinterpret_cast<uint16_t*>(sm);
    for (int x = tid; x < kBH * 32; x += NTH) {
        const int m = x >> 5, k4 = x & 31;
        put_terms(sW2, kBH, m, k4, *reinterpret_cast<const f4*>(p.q.w2 + (size_t)m * kBH + 4 * k4));
    }

    // ---- trunk: out = ReLU(W2 h + b2) of row j (three-term bf16 MFMA, as the heads), the value head, then
    //      out as the heads' B fragments: bf[c][s][t] = term t of (out[2s][0..3], out[2s+1][0..3])
    // L1: layer 1 of both tiles in one pass over the k-steps (each W1 fragment loaded once for both)
    f4 hl[L1 ? NC : 1][8];
    if constexpr (L1) {
        const int S = p.Kp / 32;
        const int x4 = p.x_stride >> 2;
        const size_t tsz = (size_t)kBH * p.Kp;
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int mt = 0; mt < 8; mt++) hl[c][mt] = (f4){0, 0, 0, 0};
        for (int s = 0; s < S; s++) {
            const int d0 = 8 * s + 2 * g4;
            u4v xb[NC];
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const uint32_t* xr = reinterpret_cast<const uint32_t*>(p.x + (size_t)rc[c] * p.x_stride);
                const uint32_t x0 = d0 < x4 ? xr[d0] : 0u, x1 = d0 + 1 < x4 ? xr[d0 + 1] : 0u;
                xb[c][0] = pack_i((int8_t)x0, (int8_t)(x0 >> 8));
                xb[c][1] = pack_i((int8_t)(x0 >> 16), (int8_t)(x0 >> 24));
                xb[c][2] = pack_i((int8_t)x1, (int8_t)(x1 >> 8));
                xb[c][3] = pack_i((int8_t)(x1 >> 16), (int8_t)(x1 >> 24));
            }
#pragma unroll
            for (int mt = 0; mt < 8; mt++) {
                const uint16_t* wp = p.w1s + (size_t)(16 * mt + j) * p.Kp + 32 * s + 8 * g4;
#pragma unroll
                for (int t = 0; t < 3; t++) {
                    const u4v wf = *reinterpret_cast<const u4v*>(wp + t * tsz);
#pragma unroll
                    for (int c = 0; c < NC; c++) hl[c][mt] = mfma_bf16(wf, xb[c], hl[c][mt]);
                }
            }
        }
    }
    __syncthreads();  // W2 staged
    u4v bf[NC][4][3];
    float value[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) {
        // layer-1 pre-activations in the trunk's B layout: h[kt][q] = h1[row j of tile c][16 kt + 4 g4 + q]
        float h[8][4];
        if constexpr (!L1) {
            f4 hv[8];
            if (p.P) {
                // compact acceptor rows: base + the owned cores' P rows in core order (= k_bdqn_l1_gather)
                const long long e = rc[c] / p.N;
                const int a1 = virt[c] ? -1 : (int)(rc[c] - e * p.N) + 1;  // the common row: no owned core
#pragma unroll
                for (int kt = 0; kt < 8; kt++) hv[kt] = *reinterpret_cast<const f4*>(p.base + 16 * kt + 4 * g4);
                const int8_t* own = p.core_owner + (size_t)e * p.C;
                const float* prow = p.P + (size_t)e * p.C * kBH + 4 * g4;
                for (int c4 = 0; c4 < p.C; c4 += 4) {
                    uint32_t ow;
                    if ((p.C & 3) == 0) {
                        ow = *reinterpret_cast<const uint32_t*>(own + c4);
                    } else {
                        ow = 0;
                        for (int u = 0; u < 4 && c4 + u < p.C; u++) ow |= (uint32_t)(uint8_t)own[c4 + u] << (8 * u);
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        if ((int)(int8_t)(ow >> (8 * u)) == a1 && c4 + u < p.C) {
                            const float* pr = prow + (size_t)(c4 + u) * kBH;
#pragma unroll
                            for (int kt = 0; kt < 8; kt++) hv[kt] += *reinterpret_cast<const f4*>(pr + 16 * kt);
                        }
                    }
                }
            } else {
#pragma unroll
                for (int kt = 0; kt < 8; kt++) hv[kt] = *reinterpret_cast<const f4*>(p.h1 + (size_t)rc[c] * kBH + 16 * kt + 4 * g4);
            }
#pragma unroll
            for (int kt = 0; kt < 8; kt++)
#pragma unroll
                for (int q = 0; q < 4; q++) h[kt][q] = hv[kt][q];
        } else {
#pragma unroll
            for (int kt = 0; kt < 8; kt++)
#pragma unroll
                for (int q = 0; q < 4; q++) h[kt][q] = hl[c][kt][q] + p.q.b1[16 * kt + 4 * g4 + q];
        }
#pragma unroll
        for (int kt = 0; kt < 8; kt++)
#pragma unroll
            for (int q = 0; q < 4; q++) h[kt][q] = fmaxf(h[kt][q], 0.f);

        u4v hb[4][3];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                v[e] = h[2 * s][e];
                v[4 + e] = h[2 * s + 1][e];
            }
            split8(v, hb[s][0], hb[s][1], hb[s][2]);
        }
        f4 acc[8];
#pragma unroll
        for (int mt = 0; mt < 8; mt++) {
            acc[mt] = (f4){0, 0, 0, 0};
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const uint16_t* ap = sW2 + (size_t)(16 * mt + j) * kAPitch + 32 * s + 8 * g4;
                acc[mt] = mfma_split6(*reinterpret_cast<const u4v*>(ap), *reinterpret_cast<const u4v*>(ap + kBH * kAPitch),
                                      *reinterpret_cast<const u4v*>(ap + 2 * kBH * kAPitch), hb[s], acc[mt]);
            }
        }
        float out[8][4];
#pragma unroll
        for (int mt = 0; mt < 8; mt++)
#pragma unroll
            for (int q = 0; q < 4; q++) out[mt][q] = fmaxf(acc[mt][q] + p.q.b2[16 * mt + 4 * g4 + q], 0.f);
        // value head: sum over the row's 128 features (lane partials in feature order, then the 4 groups)
        float vp = 0.f;
#pragma unroll
        for (int mt = 0; mt < 8; mt++)
#pragma unroll
            for (int q = 0; q < 4; q++) vp = fmaf(p.q.wv[16 * mt + 4 * g4 + q], out[mt][q], vp);
        value[c] = rows_sum(vp) + p.q.bv[0];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                v[e] = out[2 * s][e];
                v[4 + e] = out[2 * s + 1][e];
            }
            split8(v, bf[c][s][0], bf[c][s][1], bf[c][s][2]);
        }
    }
    bool explore[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) explore[c] = p.explore && rv[c] && p.explore[row[c]] != 0;

    // ---- heads, one branch at a time: Wa rows b*n + m (m < ROWS_W; zero rows past n) in LDS as three
    //      bf16 terms in the permuted K order. The next branch's f32 rows stream into an LDS staging
    //      area by LDS-DMA (global_load_lds_dwordx4, no registers) while the current one's MFMAs run;
    //      the split into terms happens between two barriers. (NMT = 8 does not fit the staging area in
    //      160 KB: it prefetches through registers.)
    constexpr bool GLDS = 3 * ROWS_W * kAPitch * 2 + ROWS_W * 4 + ROWS_W * kBH * 4 <= 160 * 1024;
    uint16_t* sWa = reinterpret_cast<uint16_t*>(sm);                        // [3][ROWS_W][kAPitch]
    float* sba = sm + (3 * ROWS_W * kAPitch) / 2;                          // [ROWS_W]
    float* sF = sba + ROWS_W;                                               // [ROWS_W][128] f32 staging (GLDS)
    constexpr int PF = GLDS ? 1 : (ROWS_W * 32 + NTH - 1) / NTH;            // f4 per thread per branch (registers)
    f4 pf[PF];
    auto fetch = [&](int b) {  // branch b's rows: LDS staging (GLDS) or registers
        if constexpr (GLDS) {
            typedef __attribute__((address_space(3))) void* lds_vp;
            typedef __attribute__((address_space(1))) void* glb_vp;
            // wave-instruction i: rows 2i, 2i + 1 (1 KB, lane-linear); rows past n read row n - 1 (zeroed at the split)
            for (int i = w; i < ROWS_W / 2; i += kActWaves) {
                const int m = 2 * i + (lane >> 5), mc = m < n ? m : n - 1;
                const float* src = p.q.wa + ((size_t)b * n + mc) * kBH + 4 * (lane & 31);
                __builtin_amdgcn_global_load_lds((glb_vp)src, (lds_vp)(sF + 256 * i), 16, 0, 0);
            }
        } else {
#pragma unroll
            for (int u = 0; u < PF; u++) {
                const int x = tid + u * NTH;
                const int m = x >> 5, k4 = x & 31;
                pf[u] = (x < ROWS_W * 32 && m < n) ? *reinterpret_cast<const f4*>(p.q.wa + ((size_t)b * n + m) * kBH + 4 * k4)
                                                   : (f4){0, 0, 0, 0};
            }
        }
    };
    __syncthreads();  // everyone is done with W2 (the staging area overlaps it)
    fetch(0);
    const float inv_n = 1.0f / (float)n;
    for (int b = 0; b < A; b++) {
        // branch b's rows have landed (LDS-DMA completion is counted by vmcnt: the compiler drains it with
        // s_waitcnt vmcnt(0) lgkmcnt(0) right before this barrier, checked in the k_bdqn_act<7, false> ISA);
        // everyone is done with the previous branch's terms
        __syncthreads();
        if constexpr (GLDS) {
            static_assert(NTH % 32 == 0, "a thread keeps its hidden-unit group across rows");
            const int k4 = tid & 31;  // the same 4 hidden units (and term positions) for every row it splits
#pragma unroll
            for (int m = tid >> 5; m < ROWS_W; m += NTH / 32) {
                const f4 v4 = m < n ? *reinterpret_cast<const f4*>(sF + m * kBH + 4 * k4) : (f4){0, 0, 0, 0};
                put_terms(sWa, ROWS_W, m, k4, v4);
            }
        } else {
#pragma unroll
            for (int u = 0; u < PF; u++) {
                const int x = tid + u * NTH;
                if (x < ROWS_W * 32) put_terms(sWa, ROWS_W, x >> 5, x & 31, pf[u]);
            }
        }
        if (tid < ROWS_W) sba[tid] = tid < n ? p.q.ba[(size_t)b * n + tid] : 0.f;
        __syncthreads();
        if (b + 1 < A) fetch(b + 1);
        f4 acc[NC][NMT];
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int mt = 0; mt < NMT; mt++) acc[c][mt] = (f4){0, 0, 0, 0};
#pragma unroll
        for (int mt = 0; mt < NMT; mt++) {
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const uint16_t* ap = sWa + (size_t)(16 * mt + j) * kAPitch + 32 * s + 8 * g4;
                const u4v a1 = *reinterpret_cast<const u4v*>(ap);
                const u4v a2 = *reinterpret_cast<const u4v*>(ap + ROWS_W * kAPitch);
                const u4v a3 = *reinterpret_cast<const u4v*>(ap + 2 * ROWS_W * kAPitch);
#pragma unroll
                for (int c = 0; c < NC; c++) acc[c][mt] = mfma_split6(a1, a2, a3, bf[c][s], acc[c][mt]);
            }
        }
#pragma unroll
        for (int c = 0; c < NC; c++) {
            // q = (value + adv) - mean(adv) over the branch's n actions; the first maximum
            // (lane (j, g4) holds actions 16 mt + 4 g4 + q of row j, increasing in (mt, q))
            // (tiles mt < NMT - 1 hold only valid actions: launch_bdqn_act instantiates NMT = ceil(n / 16)
            //  exactly, so n > 16 (NMT - 1); only the last tile is masked)
            float adv[NMT][4];
            float sum = 0.f;
#pragma unroll
            for (int mt = 0; mt < NMT; mt++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int m = 16 * mt + 4 * g4 + q;
                    adv[mt][q] = acc[c][mt][q] + sba[m];
                    if (mt < NMT - 1 || m < n) sum += adv[mt][q];
                }
            const float mean = rows_sum(sum) * inv_n;
            float best = -INFINITY;
            int bidx = 0x7fffffff;
            if constexpr (NMT >= 2) {
                // the lane's first action (4 g4 < 16 < n) starts the scan, as the first valid one
                best = (value[c] + adv[0][0]) - mean;
                bidx = 4 * g4;
            }
#pragma unroll
            for (int mt = 0; mt < NMT; mt++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int m = 16 * mt + 4 * g4 + q;
                    const float qv = (value[c] + adv[mt][q]) - mean;
                    if constexpr (NMT >= 2) {
                        if ((mt > 0 || q > 0) && (mt < NMT - 1 || m < n) && qv > best) {
                            best = qv;
                            bidx = m;
                        }
                    } else if (m < n && (qv > best || bidx == 0x7fffffff)) {
                        best = qv;
                        bidx = m;
                    }
                }
            // across the 4 lane groups: the larger q, ties to the smaller index
#pragma unroll
            for (int sh = 16; sh <= 32; sh <<= 1) {
                const float ob = __shfl_xor(best, sh);
                const int oi = __shfl_xor(bidx, sh);
                if (ob > best || (ob == best && oi < bidx)) {
                    best = ob;
                    bidx = oi;
                }
            }
            if (rv[c] && g4 == (b & 3)) {
                const int8_t act = explore[c] ? p.rnd[(size_t)row[c] * A + b] : (int8_t)bidx;
                p.action[(size_t)row[c] * A + b] = act;
            }
            if (virt[c] && g4 == (b & 3)) p.common[b] = (int8_t)bidx;  // the common row's greedy action
        }
    }
}

size_t bdqn_act_lds(int nmt) {
    const size_t rows = (size_t)16 * nmt;
    size_t heads = sizeof(uint16_t) * 3 * rows * kAPitch + sizeof(float) * rows;
    if (heads + sizeof(float) * rows * kBH <= 160 * 1024) heads += sizeof(float) * rows * kBH;  // f32 staging (GLDS)
    const size_t trunk = sizeof(uint16_t) * 3 * (size_t)kBH * kAPitch;
    return heads > trunk ? heads : trunk;
}

hipError_t launch_bdqn_w1split(const float* w1, int seg, int segs, int Dp, uint16_t* out, hipStream_t st) {
    const long long total = (long long)kBH * segs * Dp;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(k_bdqn_w1split, dim3(blocks), dim3(256), 0, st, w1, seg, segs, Dp, out);
    return hipGetLastError();
}

hipError_t launch_bdqn_l1_base(const float* w1, const float* b1, int D, int C, float* cF, float* base, hipStream_t st) {
    hipLaunchKernelGGL(k_bdqn_l1_cf, dim3(kBH, C), dim3(256), 0, st, w1, D, C, cF);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bdqn_l1_base, dim3(1), dim3(kBH), 0, st, cF, b1, C, base);
    return hipGetLastError();
}

hipError_t launch_bdqn_l1_compact(const BdqnL1Compact& p, hipStream_t st) {
    if (p.Dp > 32 * kL1MaxSteps || (p.Dp & 31)) return hipErrorInvalidValue;
    const long long rtiles = (p.E + 15) / 16;
    const long long chunks = (rtiles + kL1TilesPerWave - 1) / kL1TilesPerWave;
    const long long waves = chunks * p.C * 8;
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    switch (p.Dp / 32) {
#define MS_L1_CASE(S) \
    case S: hipLaunchKernelGGL((k_bdqn_l1_cores<S>), dim3(blocks), dim3(256), 0, st, p); break;
        MS_L1_CASE(1) MS_L1_CASE(2) MS_L1_CASE(3) MS_L1_CASE(4) MS_L1_CASE(5) MS_L1_CASE(6) MS_L1_CASE(7)
        MS_L1_CASE(8)
#undef MS_L1_CASE
        default: return hipErrorInvalidValue;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !p.h1) return e;  // (h1 NULL: the act kernel sums the P rows itself)
    const long long thr = p.E * p.N * 32;
    hipLaunchKernelGGL(k_bdqn_l1_gather, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_bdqn_act(const BdqnAct& p, hipStream_t st) {
    const int nmt = (p.q.n + 15) / 16;
    const long long rpb = 16 * kActWaves * kActTiles;  // rows per block
    const unsigned blocks = (unsigned)((p.rows + (p.list ? 1 : 0) + rpb - 1) / rpb);
    if (p.list) {
        if (p.N > 64) return hipErrorInvalidValue;
        hipError_t e;
        const long long E = p.rows / p.N;
        hipLaunchKernelGGL(k_bdqn_own_mask, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, st, p, p.own_mask);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(k_bdqn_own_list, dim3((unsigned)((p.rows + kOwnListThreads - 1) / kOwnListThreads)),
                           dim3(kOwnListThreads), 0, st, p,
                           (const unsigned long long*)p.own_mask, const_cast<int32_t*>(p.list),
                           const_cast<int32_t*>(p.n_owning));
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const bool l1 = p.h1 == nullptr && p.P == nullptr;
#define MS_BDQN_CASE(T)                                                                                  \
    if (nmt <= T) {                                                                                      \
        const size_t lds = bdqn_act_lds(T);                                                              \
        if (l1)                                                                                          \
            hipLaunchKernelGGL((k_bdqn_act<T, true>), dim3(blocks), dim3(64 * kActWaves), lds, st, p);   \
        else                                                                                             \
            hipLaunchKernelGGL((k_bdqn_act<T, false>), dim3(blocks), dim3(64 * kActWaves), lds, st, p);  \
        hipError_t e = hipGetLastError();                                                                \
        if (e != hipSuccess || !p.list) return e;                                                        \
        hipLaunchKernelGGL(k_bdqn_common_fill, dim3((unsigned)((p.rows + 255) / 256)), dim3(256), 0, st, p,  \
                           (const unsigned long long*)p.own_mask);                                        \
        return hipGetLastError();                                                                        \
    }
    // NMT = nmt exactly: the epilogue masks only the last action tile
    MS_BDQN_CASE(1) MS_BDQN_CASE(2) MS_BDQN_CASE(3) MS_BDQN_CASE(4) MS_BDQN_CASE(5) MS_BDQN_CASE(6) MS_BDQN_CASE(7)
    MS_BDQN_CASE(8)
#undef MS_BDQN_CASE
    return hipErrorInvalidValue;
}

}  // namespace ms
