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
//   k_bdqn_l1_base    b1 + sum_c W1_c F (F = the foreign acceptor row, Agent.py:167-212);
//   k_bdqn_l1_cores   layer 1 of all N agents' aggregated acceptor rows from the compact
//   k_bdqn_l1_gather  observations: an agent's row is R_c on the cores it owns and F elsewhere, so
//                     W1 x_a + b1 = base + sum_{c owned by a} W1_c (R_c - F). P_c = W1_c (R_c - F)
//                     of every (replica, core) on v_mfma_f32_16x16x32_bf16: R_c - F is a small
//                     integer (exact in bf16) and W1 is three exact bf16 terms, so every product is
//                     exact and only the f32 accumulation rounds; then every agent row adds its
//                     owned cores' P rows in core order (deterministic);
//   k_bdqn_act        the trunk, the value head and every advantage head fused with the per-branch
//                     mean, q and first-maximum argmax, then the epsilon-greedy pick: nothing but
//                     the int8 actions leaves the kernel. Trunk and heads run on
//                     v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation; no bf16 in
//                     the q values, so a greedy action differs from the fp32 reference only where
//                     two q values are within f32 rounding). The batch is on the MFMA column axis
//                     and every layer's accumulator is the next layer's B operand unchanged (the
//                     K order permuted to match); a block of 8 waves (128 rows) stages W2, then
//                     one branch's Wa rows at a time, in LDS (register prefetch of the next
//                     branch during the current one's MFMAs). With h1 == NULL layer 1 runs in the
//                     kernel on int8 rows (the offerer / price roles).
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

// ---- base[h] = b1[h] + sum_c sum_k W1[h][c*D + k] F[k]: block h, a fixed-order tree over its 256 threads
__global__ void __launch_bounds__(256) k_bdqn_l1_base(const float* __restrict__ w1, const float* __restrict__ b1, int D,
                                                      int C, float* __restrict__ base) {
    __shared__ float red[256];
    const int h = blockIdx.x, t = threadIdx.x;
    const int K = C * D;
    float s = 0.f;
    for (int i = t; i < K; i += 256) s = fmaf(w1[(size_t)h * K + i], (float)foreign(i % D, D), s);
    red[t] = s;
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
        if (t < d) red[t] += red[t + d];
        __syncthreads();
    }
    if (t == 0) base[h] = b1[h] + red[0];
}

// ---- layer 1 from compact observations, two passes.
//      k_bdqn_l1_cores: P[e][c] = W1_c (R_ec - F) for every (replica, core). A wave owns one (core,
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
    const int C = p.C, D = p.D, Dp = p.Dp;
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
    for (long long rt = t0; rt < t1; rt++) {
        const long long e = rt * 16 + i;
        const bool ev = e < p.E;
        const uint32_t* row = reinterpret_cast<const uint32_t*>(p.core_rows + ((size_t)(ev ? e : 0) * C + c) * p.stride);
        uint32_t xw[S][2];
#pragma unroll
        for (int s = 0; s < S; s++) {
            const int d0 = 8 * s + 2 * g4;
            xw[s][0] = d0 < stride4 ? row[d0] : 0u;
            xw[s][1] = d0 + 1 < stride4 ? row[d0 + 1] : 0u;
        }
        f4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < S; s++) {
            const int k0 = 32 * s + 8 * g4;
            u4v xb;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint32_t dw = xw[s][t >> 1];
                const int sh = 16 * (t & 1);
                const int ka = k0 + 2 * t, kb = ka + 1;
                const int va = ka < D ? (int)(int8_t)(dw >> sh) - foreign(ka, D) : 0;
                const int vb = kb < D ? (int)(int8_t)(dw >> (sh + 8)) - foreign(kb, D) : 0;
                xb[t] = pack_i(va, vb);
            }
            acc = mfma_bf16(aw[s][0], xb, acc);
            acc = mfma_bf16(aw[s][1], xb, acc);
            acc = mfma_bf16(aw[s][2], xb, acc);
        }
        // lane (replica i, g4) holds P_c[hidden 16 ht + 4 g4 + q] of replica e
        if (ev) *reinterpret_cast<f4*>(p.P + ((size_t)e * C + c) * kBH + 16 * ht + 4 * g4) = acc;
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

// ---- the fused trunk + heads + argmax. Block = 8 waves x 16 rows; lane (j, g4): row j of its wave's
//      tile, k-group / accumulator-row group g4.
constexpr int kActWaves = 8;

template <int NMT, bool L1>
__global__ void __launch_bounds__(64 * kActWaves) k_bdqn_act(BdqnAct p) {
    constexpr int ROWS_W = 16 * NMT;                   // staged Wa rows per branch
    constexpr int PF = (ROWS_W * 32 + 64 * kActWaves - 1) / (64 * kActWaves);  // f4 per thread per branch
    extern __shared__ __align__(16) float sm[];        // [128][kBPitch] W2, then [ROWS_W][kBPitch] Wa + ba
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int j = lane & 15, g4 = lane >> 4;
    const int n = p.q.n, A = p.q.ac_dim;
    const long long row0 = ((long long)blockIdx.x * kActWaves + w) * 16;
    const long long row = row0 + j;
    const bool rv = row < p.rows;
    const long long rc = rv ? row : p.rows - 1;

    // stage W2 (rows m, pitch kBPitch)
    for (int x = tid; x < kBH * 32; x += 64 * kActWaves) {
        const int m = x >> 5, k4 = x & 31;
        *reinterpret_cast<f4*>(sm + m * kBPitch + 4 * k4) = *reinterpret_cast<const f4*>(p.q.w2 + (size_t)m * kBH + 4 * k4);
    }

    // ---- layer-1 pre-activations in the trunk's B layout: h[kt][q] = h1[row j][16 kt + 4 g4 + q]
    float h[8][4];
    if constexpr (!L1) {
#pragma unroll
        for (int kt = 0; kt < 8; kt++) {
            const f4 v = *reinterpret_cast<const f4*>(p.h1 + (size_t)rc * kBH + 16 * kt + 4 * g4);
#pragma unroll
            for (int q = 0; q < 4; q++) h[kt][q] = v[q];
        }
    } else {
        // W1 x on the bf16 MFMA: int8 inputs exact, W1 three exact bf16 terms; D layout = B layout
        const int S = p.Kp / 32;
        const int x4 = p.x_stride >> 2;
        const uint32_t* xr = reinterpret_cast<const uint32_t*>(p.x + (size_t)rc * p.x_stride);
        const size_t tsz = (size_t)kBH * p.Kp;
        f4 acc1[8];
#pragma unroll
        for (int mt = 0; mt < 8; mt++) acc1[mt] = (f4){0, 0, 0, 0};
        for (int s = 0; s < S; s++) {
            const int d0 = 8 * s + 2 * g4;
            const uint32_t x0 = d0 < x4 ? xr[d0] : 0u, x1 = d0 + 1 < x4 ? xr[d0 + 1] : 0u;
            u4v xb;
            xb[0] = pack_i((int8_t)x0, (int8_t)(x0 >> 8));
            xb[1] = pack_i((int8_t)(x0 >> 16), (int8_t)(x0 >> 24));
            xb[2] = pack_i((int8_t)x1, (int8_t)(x1 >> 8));
            xb[3] = pack_i((int8_t)(x1 >> 16), (int8_t)(x1 >> 24));
#pragma unroll
            for (int mt = 0; mt < 8; mt++) {
                const uint16_t* wp = p.w1s + (size_t)(16 * mt + j) * p.Kp + 32 * s + 8 * g4;
#pragma unroll
                for (int t = 0; t < 3; t++) acc1[mt] = mfma_bf16(*reinterpret_cast<const u4v*>(wp + t * tsz), xb, acc1[mt]);
            }
        }
#pragma unroll
        for (int kt = 0; kt < 8; kt++)
#pragma unroll
            for (int q = 0; q < 4; q++) h[kt][q] = acc1[kt][q] + p.q.b1[16 * kt + 4 * g4 + q];
    }
#pragma unroll
    for (int kt = 0; kt < 8; kt++)
#pragma unroll
        for (int q = 0; q < 4; q++) h[kt][q] = fmaxf(h[kt][q], 0.f);
    __syncthreads();

    // ---- trunk: out[mt][q] = ReLU(W2 h + b2)[16 mt + 4 g4 + q] of row j
    float out[8][4];
    {
        f4 acc[8];
#pragma unroll
        for (int mt = 0; mt < 8; mt++) acc[mt] = (f4){0, 0, 0, 0};
#pragma unroll
        for (int kt = 0; kt < 8; kt++) {
#pragma unroll
            for (int mt = 0; mt < 8; mt++) {
                const f4 a4 = *reinterpret_cast<const f4*>(sm + (16 * mt + j) * kBPitch + 16 * kt + 4 * g4);
#pragma unroll
                for (int q = 0; q < 4; q++) acc[mt] = mfma4(a4[q], h[kt][q], acc[mt]);
            }
        }
#pragma unroll
        for (int mt = 0; mt < 8; mt++)
#pragma unroll
            for (int q = 0; q < 4; q++) out[mt][q] = fmaxf(acc[mt][q] + p.q.b2[16 * mt + 4 * g4 + q], 0.f);
    }
    // value head: sum over the row's 128 features (lane partials in feature order, then the 4 groups)
    float vp = 0.f;
#pragma unroll
    for (int mt = 0; mt < 8; mt++)
#pragma unroll
        for (int q = 0; q < 4; q++) vp = fmaf(p.q.wv[16 * mt + 4 * g4 + q], out[mt][q], vp);
    const float value = rows_sum(vp) + p.q.bv[0];
    const bool explore = p.explore && rv && p.explore[row] != 0;

    // ---- heads, one branch at a time: Wa rows b*n + m (m < ROWS_W; zero rows past n) in LDS
    float* sWa = sm;                       // [ROWS_W][kBPitch]
    float* sba = sm + ROWS_W * kBPitch;    // [ROWS_W]
    f4 pf[PF];
    float pfb = 0.f;
    auto fetch = [&](int b) {  // branch b's rows into registers
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int x = tid + u * 64 * kActWaves;
            const int m = x >> 5, k4 = x & 31;
            pf[u] = (x < ROWS_W * 32 && m < n) ? *reinterpret_cast<const f4*>(p.q.wa + ((size_t)b * n + m) * kBH + 4 * k4)
                                               : (f4){0, 0, 0, 0};
        }
        pfb = (tid < ROWS_W && tid < n) ? p.q.ba[(size_t)b * n + tid] : 0.f;
    };
    fetch(0);
    const float inv_n = 1.0f / (float)n;
    for (int b = 0; b < A; b++) {
        __syncthreads();  // everyone is done with the previous branch's rows (and with W2)
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int x = tid + u * 64 * kActWaves;
            if (x < ROWS_W * 32) *reinterpret_cast<f4*>(sWa + (x >> 5) * kBPitch + 4 * (x & 31)) = pf[u];
        }
        if (tid < ROWS_W) sba[tid] = pfb;
        __syncthreads();
        if (b + 1 < A) fetch(b + 1);
        f4 acc[NMT];
#pragma unroll
        for (int mt = 0; mt < NMT; mt++) acc[mt] = (f4){0, 0, 0, 0};
#pragma unroll
        for (int kt = 0; kt < 8; kt++) {
#pragma unroll
            for (int mt = 0; mt < NMT; mt++) {
                const f4 a4 = *reinterpret_cast<const f4*>(sWa + (16 * mt + j) * kBPitch + 16 * kt + 4 * g4);
#pragma unroll
                for (int q = 0; q < 4; q++) acc[mt] = mfma4(a4[q], out[kt][q], acc[mt]);
            }
        }
        // q = (value + adv) - mean(adv) over the branch's n actions; the first maximum
        // (lane (j, g4) holds actions 16 mt + 4 g4 + q of row j, increasing in (mt, q))
        float adv[NMT][4];
        float sum = 0.f;
#pragma unroll
        for (int mt = 0; mt < NMT; mt++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int m = 16 * mt + 4 * g4 + q;
                adv[mt][q] = acc[mt][q] + sba[m];
                if (m < n) sum += adv[mt][q];
            }
        const float mean = rows_sum(sum) * inv_n;
        float best = -INFINITY;
        int bidx = 0x7fffffff;
#pragma unroll
        for (int mt = 0; mt < NMT; mt++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int m = 16 * mt + 4 * g4 + q;
                const float qv = (value + adv[mt][q]) - mean;
                if (m < n && (qv > best || bidx == 0x7fffffff)) {
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
        if (rv && g4 == (b & 3)) {
            const int8_t act = explore ? p.rnd[(size_t)row * A + b] : (int8_t)bidx;
            p.action[(size_t)row * A + b] = act;
        }
    }
}

size_t bdqn_act_lds(int nmt) {
    const size_t heads = sizeof(float) * ((size_t)16 * nmt * kBPitch + 16 * nmt);
    const size_t trunk = sizeof(float) * (size_t)kBH * kBPitch;
    return heads > trunk ? heads : trunk;
}

hipError_t launch_bdqn_w1split(const float* w1, int seg, int segs, int Dp, uint16_t* out, hipStream_t st) {
    const long long total = (long long)kBH * segs * Dp;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(k_bdqn_w1split, dim3(blocks), dim3(256), 0, st, w1, seg, segs, Dp, out);
    return hipGetLastError();
}

hipError_t launch_bdqn_l1_base(const float* w1, const float* b1, int D, int C, float* base, hipStream_t st) {
    hipLaunchKernelGGL(k_bdqn_l1_base, dim3(kBH), dim3(256), 0, st, w1, b1, D, C, base);
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
    if (e != hipSuccess) return e;
    const long long thr = p.E * p.N * 32;
    hipLaunchKernelGGL(k_bdqn_l1_gather, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_bdqn_act(const BdqnAct& p, hipStream_t st) {
    const int nmt = (p.q.n + 15) / 16;
    const unsigned blocks = (unsigned)((p.rows + 16 * kActWaves - 1) / (16 * kActWaves));
    const bool l1 = p.h1 == nullptr;
#define MS_BDQN_CASE(T)                                                                                  \
    if (nmt <= T) {                                                                                      \
        const size_t lds = bdqn_act_lds(T);                                                              \
        if (l1)                                                                                          \
            hipLaunchKernelGGL((k_bdqn_act<T, true>), dim3(blocks), dim3(64 * kActWaves), lds, st, p);   \
        else                                                                                             \
            hipLaunchKernelGGL((k_bdqn_act<T, false>), dim3(blocks), dim3(64 * kActWaves), lds, st, p);  \
        return hipGetLastError();                                                                        \
    }
    MS_BDQN_CASE(1) MS_BDQN_CASE(3) MS_BDQN_CASE(7) MS_BDQN_CASE(8)
#undef MS_BDQN_CASE
    return hipErrorInvalidValue;
}

}  // namespace ms
