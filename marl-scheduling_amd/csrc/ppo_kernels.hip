// ppo_kernels.hip — fused PPO loss gradient for groups of 16-wide actor-critics on gfx950.
//
// One K-epoch step of PPO.update (PPOmodules.py:144-168) needs, per group g,
// d/dθ of  mean_r[ -min(ratio*adv, clamp(ratio)*adv) ] + 0.5*mean_r[(V-G)^2] - 0.01*mean_r[H]
// over R = T*E rows (torch Categorical semantics: probs renormalised,
// logits = log(clamp(p, eps, 1-eps)), entropy -sum(logits*p)). k_ppo_grad
// computes it in one pass over the int8 rollout buffer.
//
// Work split: a block is 4 waves of one group sharing the group's weights in
// LDS; each wave walks a contiguous range of 16-row tiles and accumulates its
// own partial gradient. Per tile:
//  * forward on v_mfma_f32_16x16x4_f32 with the batch on the MFMA column (lane)
//    axis, so every layer's accumulator is the next layer's B operand. Layer 1
//    takes its B operand straight from the prefetched observation dwords
//    (k order permuted to match: step (m, b) = byte b of dword g4+4m); the
//    weights are read with the same permutation (ds_read_b128);
//  * softmax / renormalisation / clamped log / entropy, the per-row loss
//    derivatives (torch.minimum splits ties, clamp backward is inclusive) and
//    the backward pass through the tanh layers, on the accumulator layout;
//  * weight gradients as MFMAs with K = rows. Their operands go through small
//    LDS transposes whose pitch (20 floats) and row order make both the writes
//    and the ds_read_b128 reads bank-conflict free. Layer 1's input tile is
//    staged with byte D set to 1, so column D of dW1 is the bias gradient.
// Each wave writes one partial gradient vector; k_ppo_reduce sums them in a
// fixed order (deterministic) into the torch .grad tensors.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "../../include/marlsched.h"
#include "ms_common.h"
#include "ms_ppo.h"

namespace ms {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

__device__ __forceinline__ float xsum16(float v) {  // sum over the 16 lanes sharing lane>>4
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    return v;
}
__device__ __forceinline__ float xsum4g(float v) { return rows_sum(v); }  // sum over lanes j, j+16, j+32, j+48
__device__ __forceinline__ float xmax4g(float v) { return rows_max(v); }

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

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma_bf16(const u4v& a, const u4v& b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                   0);
}
// bf16 (upper half of the f32 bits) of two floats packed into one dword
__device__ __forceinline__ uint32_t pack_hi(float lo, float hi) {
    return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);  // one v_perm_b32
}
__device__ __forceinline__ float trunc_bf16(float x) { return __uint_as_float(__float_as_uint(x) & 0xffff0000u); }

// 8 floats as three bf16 fragments with v = hi + mid + lo exactly (truncation leaves exact residuals)
__device__ __forceinline__ void split3(const float (&v)[8], u4v& hi, u4v& mid, u4v& lo) {
#pragma unroll
    for (int d = 0; d < 4; d++) {
        float h[2], m[2], l[2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
            h[t] = trunc_bf16(v[2 * d + t]);
            const float r = v[2 * d + t] - h[t];
            m[t] = trunc_bf16(r);
            l[t] = r - m[t];
        }
        hi[d] = pack_hi(h[0], h[1]);
        mid[d] = pack_hi(m[0], m[1]);
        lo[d] = pack_hi(l[0], l[1]);
    }
}

// int8 values (exact in bf16) packed in pairs
__device__ __forceinline__ uint32_t pack_i8(int a, int b) { return pack_hi((float)a, (float)b); }
__device__ __forceinline__ u4v bytes_to_bf16(uint32_t d0, uint32_t d1) {
    u4v r;
    r[0] = pack_i8((int8_t)d0, (int8_t)(d0 >> 8));
    r[1] = pack_i8((int8_t)(d0 >> 16), (int8_t)(d0 >> 24));
    r[2] = pack_i8((int8_t)d1, (int8_t)(d1 >> 8));
    r[3] = pack_i8((int8_t)(d1 >> 16), (int8_t)(d1 >> 24));
    return r;
}

constexpr int kCommonSeg = 512;   // rows scanned per segment of the common-row path
#ifndef MS_XCD_MAP
#define MS_XCD_MAP 1
#endif
#ifndef MS_OWN_SEG
#define MS_OWN_SEG 512
#endif
template <int MODE>
constexpr int seg_rows() { return MODE == 2 ? MS_OWN_SEG : kCommonSeg; }  // (2 = kOwnerRow)
constexpr int kScanDepth = 1;     // 64-row scan steps in flight (2 spills registers at <4, 2>: slower)
#ifndef MS_OWN_DEPTH
#define MS_OWN_DEPTH 1
#endif
constexpr int kScanDepthOwn = MS_OWN_DEPTH;  // the same for compact rows (no row chunks in the scan registers)

template <bool B>
struct BoolC {
    static constexpr bool value = B;
};

// kernel modes: every row on its own; rows equal to one common row (found by comparing the rows, or
// from the core owners of compact acceptor observations); keyed rows (the backward and the forward
// of a group's distinct rows, k_key_scan sums the rows' loss derivatives in between)
enum GradMode { kPlain = 0, kCommonRow = 1, kOwnerRow = 2, kKeyBack = 3, kKeyFwd = 4, kMaskRow = 5, kCommonFwd = 6 };
constexpr int kX1 = 16;  // mode bit: the last action tile has exactly one action (k_ppo_grad)
// kMaskRow: compact acceptor rows of many groups (the divided acceptors), the common rows already
// summed by k_own_scan / k_own_common: each wave runs the tiles of the rows its group's own-row mask
// lists, and one wave per group the common rows' virtual tile. kCommonFwd: the forward of the
// common row of every group (k_own_scan's table).
constexpr int kMaskList = 1024 + 64;  // LDS list of one wave in kMaskRow: < 16 carried + 32 mask words

#ifdef MS_GRAD_PROBE
// Probe build only (tools/grad_probe.py): per wave of the last common/owner-row launch, s_memrealtime
// at entry, after the scan, at exit, and the rows the scan listed for the tiles.
constexpr int kGradProbeWaves = 1 << 15;
__device__ unsigned long long g_grad_probe[kGradProbeWaves][4];
#endif

// (The 16-wide layers stay on the f32 MFMA: a three-term bf16 form of them measured slower, 2519 -> 2646 us
// per offer-gradient call, profiles/r5m)

template <int NQ, int NT, int MODEX>
struct GradLds {
    static constexpr int MODE = MODEX & 15;  // (bit 4: kX1, see k_ppo_grad)
    static constexpr bool CM = MODE == kCommonRow || MODE == kOwnerRow;
    static constexpr bool ML = MODE == kMaskRow;
    static constexpr int S1 = (NQ + 1) / 2;           // 32-input k-steps of layer 1 (16*NQ inputs)
    static constexpr int W1B = 32 * S1 + 8;           // bf16 pitch of a split W1 row (+16 B: no conflicts)
    static constexpr int XPD = (NQ & 1) ? 4 * NQ + 6 : 4 * NQ + 2;  // staged input row pitch (dwords)
    static constexpr int TP = 20;                     // 16-row transpose pitch (floats)
    static constexpr int TP2 = 36;                    // 32-row transpose pitch (floats)
    static constexpr int NTR = NT + 1;               // 16-row transposes live at once (three phases per tile)
    // block: split W1 / C1 [2][3][16][W1B] bf16, then W2, C2, W3 and the biases (floats)
    static constexpr int w1s_floats = 2 * 3 * 16 * W1B / 2;
    static constexpr int shared_floats = w1s_floats + 2 * 256 + 256 * NT + 16 * 5 + 16 * NT + 4;
    // per wave: d1 / e1 transposes over a tile pair, the per-tile transposes, 32 staged input rows
    // (common-row path: the common row's clamped logs, V, entropy, the list of the other rows,
    //  and the wave's int64 fixed-point sums of d min(surr)/d ratio * ratio per action [16*NT])
    static constexpr int CMF = CM ? 16 * NT + 4 + seg_rows<MODE>() + 64 + 2 * 16 * NT : (ML ? kMaskList : 0);
    static constexpr int wave_floats = 2 * 16 * TP2 + NTR * 16 * TP + 32 * XPD + CMF;
    // waves per block: 4 when they fit the 160 KB of LDS, else 2 (each wave then walks two chunks)
    static constexpr int WPB = shared_floats + 4 * wave_floats <= 40960 ? 4 : 2;
    static constexpr int lds_floats = shared_floats + WPB * wave_floats;
};

// NQ = 16-wide input tiles with 16*NQ > D, NT = ceil(A/16) action tiles. A block owns 4 chunks
// of one group and has L::WPB waves.
template <int NQ, int NT, int MODEX>
__global__ void __launch_bounds__((64 * GradLds<NQ, NT, MODEX>::WPB), ((NQ * NT >= 32) ? 1 : 2)) k_ppo_grad(PpoArgs p) {
    using L = GradLds<NQ, NT, MODEX>;
    constexpr int MODE = MODEX & 15;
    // kX1: the last action tile holds one action (A = 16 (NT - 1) + 1, e.g. C + 1 = 17 or O + 1 = 49 at
    // cfg4): its layer-3 row, backward term and weight gradient run on the VALU (4 FMAs per lane and a
    // sum over the row's lane groups) instead of 12 f32 MFMAs on a tile of 15 padding actions
    constexpr bool X1 = (MODEX & kX1) != 0;
    constexpr int TP = L::TP, TP2 = L::TP2, XPD = L::XPD, S1 = L::S1, W1B = L::W1B;
    constexpr int NTH = 64 * L::WPB, CPW = 4 / L::WPB;  // threads per block, chunks per wave
    // the wave index through readfirstlane: everything derived from it (chunk, tile range, row buffers)
    // is wave-uniform to the compiler and lives in scalar registers
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g4 = lane >> 4;  // MFMA k-group / C-row group
    const int j = lane & 15;   // batch row within the tile (C column)
    // XCD-aware block map: blocks b and b + 8 run on one XCD (round-robin placement, speed only), so
    // the G groups' blocks of one row range take block indices 8 apart: they run on the same XCD at
    // about the same time, and the rollout lines they share (rows [r][0..U) of states, actions,
    // log-probs, returns) come into that XCD's L2 once instead of once per group's XCD
#if MS_XCD_MAP
    const int xq = blockIdx.x >> 3;
    const int grp = xq % p.G;
    const int blk = (xq / p.G) * 8 + (blockIdx.x & 7);
    if (blk >= p.blocks_per_group) return;  // padding of the grid to whole 8-block sets (whole block)
#else
    const int grp = blockIdx.x % p.G;
    const int blk = blockIdx.x / p.G;
#endif
    const int chunk = blk * 4 + wave * CPW;
    const int D = p.D, A = p.A;
    const int u = p.unit_of_group[grp];

    extern __shared__ __align__(16) float sm[];
    uint16_t* sW1s = reinterpret_cast<uint16_t*>(sm);  // [net][hi/mid/lo][16][W1B] bf16 (zero beyond D)
    float* sW2 = sm + L::w1s_floats;    // [16][16]
    float* sC2 = sW2 + 256;             // [16][16]
    float* sW3 = sC2 + 256;             // [16*NT][16] (zero rows >= A)
    float* sb1 = sW3 + 256 * NT;        // 16
    float* sb2 = sb1 + 16;              // 16
    float* sc3 = sb2 + 16;              // 16 (critic output row)
    float* scb1 = sc3 + 16;             // 16
    float* scb2 = scb1 + 16;            // 16
    float* sb3 = scb2 + 16;             // 16*NT
    float* scb3 = sb3 + 16 * NT;        // 1 (+3 pad)
    float* sT = sm + L::shared_floats + wave * L::wave_floats;
    float* T_d1 = sT;                   // [16 features][TP2]: 32 rows of the tile pair
    float* T_e1 = sT + 16 * TP2;
    float* sT1 = sT + 2 * 16 * TP2;     // [NTR][16][TP]
    uint32_t* sX = reinterpret_cast<uint32_t*>(sT1 + L::NTR * 16 * TP);  // [32][XPD] dwords
    float* sCm = reinterpret_cast<float*>(sX + 32 * XPD);  // common-row path (L::CMF floats)

    // behind the keyed passes (key_n set), the tile path only runs the groups they could not take;
    // k_ppo_reduce skips this block's partial row for the others
    if constexpr (MODE == kPlain)
        if (p.key_n && p.key_n[grp] >= 0 && p.key_flag[grp] == 0) return;
#ifdef MS_GRAD_PROBE
    const unsigned long long probe_t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long probe_listed = 0, probe_t1 = 0;
#endif

    // ---- stage this group's weights (once per block); W1 / C1 as three exact bf16 terms
    {
        const float* W1 = p.w1 + (size_t)grp * 16 * D;
        const float* C1 = p.cw1 + (size_t)grp * 16 * D;
        for (int i = tid; i < 2 * 16 * 32 * S1; i += NTH) {
            const int net = i / (16 * 32 * S1), rem = i - net * 16 * 32 * S1;
            const int r = rem / (32 * S1), c = rem - r * (32 * S1);
            const float w = c < D ? (net ? C1 : W1)[r * D + c] : 0.f;
            const float h = trunc_bf16(w), rr = w - h, m = trunc_bf16(rr), l = rr - m;
            uint16_t* base = sW1s + net * 3 * 16 * W1B + r * W1B + c;
            base[0] = (uint16_t)(__float_as_uint(h) >> 16);
            base[16 * W1B] = (uint16_t)(__float_as_uint(m) >> 16);
            base[2 * 16 * W1B] = (uint16_t)(__float_as_uint(l) >> 16);
        }
        for (int i = tid; i < 256; i += NTH) {
            sW2[i] = p.w2[(size_t)grp * 256 + i];
            sC2[i] = p.cw2[(size_t)grp * 256 + i];
        }
        for (int i = tid; i < 256 * NT; i += NTH) {
            const int a = i >> 4;
            sW3[i] = a < A ? p.w3[((size_t)grp * A + a) * 16 + (i & 15)] : 0.f;
        }
        for (int i = tid; i < 16 * NT; i += NTH) sb3[i] = i < A ? p.b3[(size_t)grp * A + i] : 0.f;
        if (tid < 16) {
            sb1[tid] = p.b1[grp * 16 + tid] * kTanhScale;  // hidden biases pre-scaled (fast_tanh_b)
            sb2[tid] = p.b2[grp * 16 + tid] * kTanhScale;
            sc3[tid] = p.cw3[grp * 16 + tid];
            scb1[tid] = p.cb1[grp * 16 + tid] * kTanhScale;
            scb2[tid] = p.cb2[grp * 16 + tid] * kTanhScale;
        }
        if (tid == 0) scb3[0] = p.cb3[grp];
    }
    __syncthreads();
    f4 gW1[NQ], gC1[NQ], gW3[NT];
    f4 gW2 = {0, 0, 0, 0}, gC2 = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < NQ; q++) gW1[q] = gC1[q] = (f4){0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < NT; t++) gW3[t] = (f4){0, 0, 0, 0};
    float db2[4] = {0, 0, 0, 0}, cdb2[4] = {0, 0, 0, 0}, gC3[4] = {0, 0, 0, 0};
    float gW3x[4] = {0, 0, 0, 0};  // (kX1) d W3[16 (NT - 1)][4 g4 + q] over this lane's rows
    float db3[NT][4];
#pragma unroll
    for (int t = 0; t < NT; t++) db3[t][0] = db3[t][1] = db3[t][2] = db3[t][3] = 0.f;
    float cdb3 = 0.f, l_min = 0.f, l_mse = 0.f, l_ent = 0.f;
    const float eps = 1.1920928955078125e-07f;

    const int stride4 = p.stride >> 2;
    const int R = (int)p.R;
    const int tile0 = chunk * p.chunk_tiles;
    const int tile_end = min(tile0 + CPW * p.chunk_tiles, (R + 15) >> 4);
    // input byte D of every staged row reads 1 (the bias column of dW1)
    const int one_dw = D >> 2;
    const uint32_t one_bit = 1u << (8 * (D & 3));
    // compact acceptor rows: unit u = agent u / C, core u % C reads core row (r, u % C)
    constexpr bool OWNROWS = MODE == kOwnerRow || MODE == kMaskRow;  // rows are compact core rows
    const int own_c = OWNROWS ? u % p.owner_C : 0;
    const int8_t own_me = OWNROWS ? (int8_t)(u / p.owner_C + 1) : 0;
    auto row_src = [&](int r) {
        if constexpr (OWNROWS)
            return reinterpret_cast<const uint32_t*>(p.states + ((size_t)r * p.owner_C + own_c) * p.stride);
        else
            return reinterpret_cast<const uint32_t*>(p.states + ru_index(p, r, u) * p.stride);
    };
    const float zero_vs[NT][4] = {};

    // ---- forward of one 16-row tile (lane (j, g4) holds dwords 8s + 2*g4 + {0, 1} of row j as xw,
    //      byte D set to 1): hidden activations, softmax (nn.Softmax) + Categorical(probs)
    //      renormalisation, clamped logs, critic output and entropy of row j
    struct Fwd {
        float h1[4], hc1[4], h2[4], hc2[4];
        float pe[NT][4], pn[NT][4], cl[NT][4];
        float inv1, V, ent;
    };
    auto forward = [&](const uint32_t (&xw)[S1][2], Fwd& f) {
        // layer 1 on the bf16 MFMA: the int8 inputs are exact in bf16, the weights are
        // hi + mid + lo; actor and critic share the B operand
        f4 a1 = {0, 0, 0, 0}, c1 = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < S1; s++) {
            const u4v xb = bytes_to_bf16(xw[s][0], xw[s][1]);
#pragma unroll
            for (int t = 0; t < 3; t++) {
                const u4v wa = *reinterpret_cast<const u4v*>(sW1s + (0 * 3 + t) * 16 * W1B + j * W1B + 32 * s + 8 * g4);
                const u4v wc = *reinterpret_cast<const u4v*>(sW1s + (1 * 3 + t) * 16 * W1B + j * W1B + 32 * s + 8 * g4);
                a1 = mfma_bf16(wa, xb, a1);
                c1 = mfma_bf16(wc, xb, c1);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            f.h1[q] = fast_tanh_b(a1[q], sb1[4 * g4 + q]);
            f.hc1[q] = fast_tanh_b(c1[q], scb1[4 * g4 + q]);
        }
        // layer 2: B operand = layer-1 output as is; A reads W2 with k permuted (k_true = 4*g4 + s)
        f4 a2 = {0, 0, 0, 0}, c2 = {0, 0, 0, 0};
        {
            const f4 w2 = *reinterpret_cast<const f4*>(sW2 + j * 16 + 4 * g4);
            const f4 cw2 = *reinterpret_cast<const f4*>(sC2 + j * 16 + 4 * g4);
#pragma unroll
            for (int s = 0; s < 4; s++) {
                a2 = mfma4(w2[s], f.h1[s], a2);
                c2 = mfma4(cw2[s], f.hc1[s], c2);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            f.h2[q] = fast_tanh_b(a2[q], sb2[4 * g4 + q]);
            f.hc2[q] = fast_tanh_b(c2[q], scb2[4 * g4 + q]);
        }
        // actor layer 3 -> logits z[a = 16t + 4*g4 + q][row j]
        float z[NT][4];
#pragma unroll
        for (int t = 0; t < NT; t++) {
            f4 zz = {0, 0, 0, 0};
            if (X1 && t == NT - 1) {
                // action 16 t alone: W3[16 t] . h2 as this lane's 4 terms, summed over the row's lane groups
                const f4 w3 = *reinterpret_cast<const f4*>(sW3 + (16 * t) * 16 + 4 * g4);
                float pz = 0.f;
#pragma unroll
                for (int q = 0; q < 4; q++) pz = fmaf(w3[q], f.h2[q], pz);
                zz[0] = xsum4g(pz);
            } else {
                const f4 w3 = *reinterpret_cast<const f4*>(sW3 + (16 * t + j) * 16 + 4 * g4);
#pragma unroll
                for (int s = 0; s < 4; s++) zz = mfma4(w3[s], f.h2[s], zz);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) z[t][q] = zz[q] + sb3[16 * t + 4 * g4 + q];
        }
        // critic output V (one row of the last layer, summed across the 4 lane groups together with
        // the softmax denominator below)
        float vp = 0.f;
#pragma unroll
        for (int q = 0; q < 4; q++) vp = fmaf(sc3[4 * g4 + q], f.hc2[q], vp);
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (16 * t + 4 * g4 + q < A) mx = fmaxf(mx, z[t][q]);
        mx = xmax4g(mx);
        const float mx_l2e = mx * 1.4426950408889634f;
        float s0 = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                f.pe[t][q] = (16 * t + 4 * g4 + q < A) ? fast_exp_sub(z[t][q], mx_l2e) : 0.f;
                s0 += f.pe[t][q];
            }
        rows_sum2(s0, vp);
        f.V = vp + scb3[0];
        const float inv0 = __builtin_amdgcn_rcpf(s0);
        float s1 = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                f.pe[t][q] *= inv0;  // softmax output (same arithmetic as k_act)
                s1 += f.pe[t][q];
            }
        f.inv1 = __builtin_amdgcn_rcpf(xsum4g(s1));
        float ent = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                f.pn[t][q] = f.pe[t][q] * f.inv1;
                f.cl[t][q] = fast_log(fminf(fmaxf(f.pn[t][q], eps), 1.f - eps));
                if (16 * t + 4 * g4 + q < A) ent -= f.cl[t][q] * f.pn[t][q];
            }
        f.ent = ent;  // this lane's part: the row's entropy is xsum4g(f.ent) (ent_of)
    };
    auto ent_of = [&](const Fwd& f) { return xsum4g(f.ent); };

    if constexpr (MODE == kCommonFwd) {
        // the common row's forward values of this group: clamped log-probs [16*NT], V, entropy (the
        // table k_own_scan reads; the same forward as the tiles and the virtual tile)
        if (wave == 0) {
            const uint32_t* crow = reinterpret_cast<const uint32_t*>(p.common);
            uint32_t xw[S1][2];
#pragma unroll
            for (int s = 0; s < S1; s++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int cc = 8 * s + 2 * g4 + h;
                    xw[s][h] = cc < stride4 ? crow[cc] : 0u;
                }
            Fwd f;
            forward(xw, f);
            const float ent_row = ent_of(f);
            float* dst = p.own_cfwd + (size_t)grp * (16 * NT + 4);
            if (j == 0) {
#pragma unroll
                for (int t = 0; t < NT; t++)
#pragma unroll
                    for (int q = 0; q < 4; q++) dst[16 * t + 4 * g4 + q] = f.cl[t][q];
                if (g4 == 0) {
                    dst[16 * NT] = f.V;
                    dst[16 * NT + 1] = ent_row;
                }
            }
        }
        return;
    }

    // ---- one 16-row tile: forward, per-row loss derivatives, backward, weight gradients.
    //      xr = the rows' raw dwords (B-fragment layout), act/olp/G/valid = row j's scalars.
    //      VIRT: the common row's virtual tile, whose column-0 derivatives are sums over every
    //      row equal to the common row (vsum[a] = sum of d loss / d logp over those rows that took
    //      action a, vgh / vgv = summed entropy / value derivatives; zero in the other columns):
    //      the backward is linear in them, so one pass gives those rows' summed weight gradients.
    auto tile_step = [&](auto virt, const uint32_t (&xr)[S1][2], int act, float olp, float G, bool valid, int half,
                         bool pair_done, const float (&vsum)[NT][4], float vgh, float vgv) {
        constexpr bool VIRT = decltype(virt)::value;
        // wide inputs: re-read the split W1 from LDS per tile instead of holding it in registers
        if (S1 > 2) __asm__ volatile("" ::: "memory");
        uint32_t xw[S1][2];
#pragma unroll
        for (int s = 0; s < S1; s++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int cc = 8 * s + 2 * g4 + h;
                const uint32_t w = cc < stride4 ? xr[s][h] : 0u;  // bytes past the row read 0
                xw[s][h] = cc == one_dw ? (w | one_bit) : w;
                if (cc < 4 * NQ) sX[(16 * half + j) * XPD + cc] = xw[s][h];
            }
        Fwd f;
        forward(xw, f);
        const float V = f.V;
        float g_lp = 0.f, g_v, g_h;
        if (VIRT) {
            g_v = vgv;
            g_h = vgh;
        } else {
            float lp = 0.f;
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (16 * t + 4 * g4 + q < A && 16 * t + 4 * g4 + q == act) lp += f.cl[t][q];
            float ent = f.ent;
            rows_sum2(lp, ent);  // the action's log-prob and the row's entropy
            // ---- per-row loss derivatives (loss.mean() over R rows)
            const float ratio = fast_exp(lp - olp);
            const float adv = G - V;
            const float sur1 = ratio * adv;
            const float rc = fminf(fmaxf(ratio, 1.f - p.eps_clip), 1.f + p.eps_clip);
            const float sur2 = rc * adv;
            const float inr = (ratio >= 1.f - p.eps_clip && ratio <= 1.f + p.eps_clip) ? 1.f : 0.f;
            // d min(s1, s2) / d ratio (torch.minimum splits ties)
            const float dmin = sur1 < sur2 ? adv : (sur2 < sur1 ? adv * inr : 0.5f * adv + 0.5f * adv * inr);
            const float w = valid ? p.inv_R : 0.f;
            g_lp = -dmin * w * ratio;  // d loss / d logp (exp backward uses the result)
            g_v = (V - G) * w;         // 0.5 * d MSE / d V
            g_h = -0.01f * w;          // d loss / d entropy
            if (valid && g4 == 0) {
                l_min += -fminf(sur1, sur2);
                l_mse += (V - G) * (V - G);
                l_ent += ent;
            }
        }
        // d loss / d pn  -> d / d p (renormalisation) -> d / d z (softmax)
        float gz[NT][4], x1 = 0.f;
        if constexpr (VIRT) {
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int a = 16 * t + 4 * g4 + q;
                    float v = 0.f;
                    if (a < A) {
                        const float dc = vsum[t][q] - g_h * f.pn[t][q];
                        const float in = (f.pn[t][q] >= eps && f.pn[t][q] <= 1.f - eps) ? 1.f : 0.f;
                        v = dc * in * __builtin_amdgcn_rcpf(fminf(fmaxf(f.pn[t][q], eps), 1.f - eps)) -
                            g_h * f.cl[t][q];
                    }
                    gz[t][q] = v;
                    x1 += v * f.pe[t][q];
                }
        } else {
            // one row's loss touches the log-prob of its own action only: d/d pn_a of
            // g_lp * log(clamp(pn_act)) - g_h * H is (g_lp / pn_act at a = act) - g_h (in range),
            // - g_h * cl_a throughout; the one reciprocal per lane is of its copy of pn_act
            float pa = 1.f;
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int q = 0; q < 4; q++) pa = (16 * t + 4 * g4 + q == act) ? f.pn[t][q] : pa;
            const float dact = g_lp * __builtin_amdgcn_rcpf(pa);
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int a = 16 * t + 4 * g4 + q;
                    const bool in = f.pn[t][q] >= eps && f.pn[t][q] <= 1.f - eps;
                    const float d_in = (a == act ? dact : 0.f) - g_h;
                    const float v = a < A ? fmaf(-g_h, f.cl[t][q], in ? d_in : 0.f) : 0.f;
                    gz[t][q] = v;
                    x1 += v * f.pe[t][q];
                }
        }
        x1 = xsum4g(x1);
        const float inv1 = f.inv1;
        float x2 = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                gz[t][q] = (gz[t][q] - x1 * inv1) * inv1;
                x2 += gz[t][q] * f.pe[t][q];
            }
        x2 = xsum4g(x2);
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) gz[t][q] = f.pe[t][q] * (gz[t][q] - x2);

        // ---- backward through the hidden layers (same no-movement trick, transposed weights)
        f4 d2 = {0, 0, 0, 0};
        float g16 = 0.f;  // (kX1) the single action's dz of row j, on every lane of the row
#pragma unroll
        for (int t = 0; t < NT; t++) {
            if (X1 && t == NT - 1) {
                g16 = __shfl(gz[t][0], j);  // lane (j, 0) holds action 16 t
                const f4 w3 = *reinterpret_cast<const f4*>(sW3 + (16 * t) * 16 + 4 * g4);
#pragma unroll
                for (int q = 0; q < 4; q++) d2[q] = fmaf(w3[q], g16, d2[q]);
            } else {
#pragma unroll
                for (int s = 0; s < 4; s++) d2 = mfma4(sW3[(16 * t + 4 * g4 + s) * 16 + j], gz[t][s], d2);
            }
        }
        float dl2[4], dc2[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            dl2[q] = d2[q] * (1.f - f.h2[q] * f.h2[q]);
            dc2[q] = sc3[4 * g4 + q] * g_v * (1.f - f.hc2[q] * f.hc2[q]);
        }
        f4 d1 = {0, 0, 0, 0}, e1 = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 4; s++) {
            d1 = mfma4(sW2[(4 * g4 + s) * 16 + j], dl2[s], d1);
            e1 = mfma4(sC2[(4 * g4 + s) * 16 + j], dc2[s], e1);
        }
        float dl1[4], dc1[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            dl1[q] = d1[q] * (1.f - f.h1[q] * f.h1[q]);
            dc1[q] = e1[q] * (1.f - f.hc1[q] * f.hc1[q]);
        }
        // bias gradients of layers 2-3 and the critic output layer (VALU; reduced over rows at the end)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            db2[q] += dl2[q];
            cdb2[q] += dc2[q];
            gC3[q] = fmaf(g_v, f.hc2[q], gC3[q]);
#pragma unroll
            for (int t = 0; t < NT; t++) db3[t][q] += gz[t][q];
        }
        if (g4 == 0) cdb3 += g_v;

        // ---- weight gradients: batch reductions as MFMAs with K = rows. 16-row transposes:
        //      value of (feature f, row r) at T[f*TP + 4*(r%4) + r/4], so lane (j, g4) reads rows
        //      g4, g4+4, g4+8, g4+12 of feature j with one ds_read_b128 (k step s = row g4 + 4s).
        //      d1 / e1 go to the tile pair's 32-row transposes (row 16*half + j at T2[f*TP2 + row]).
        //      Three phases share the transpose space (L::NTR arrays): dW2, dC2, then dW3.
        float* T_d2 = sT1;
        float* T_h1 = sT1 + 1 * 16 * TP;
        float* T_e2 = sT1;
        float* T_k1 = sT1 + 1 * 16 * TP;
        float* T_h2 = sT1;
        float* T_gz = sT1 + 1 * 16 * TP;
        const int pr = 4 * (j & 3) + (j >> 2);  // this lane's row position
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int fo = (4 * g4 + q) * TP + pr;
            T_d2[fo] = dl2[q];
            T_h1[fo] = f.h1[q];
            const int f2 = (4 * g4 + q) * TP2 + 16 * half + j;
            T_d1[f2] = dl1[q];
            T_e1[f2] = dc1[q];
        }
        if (half == 0 && pair_done) {  // odd tile count: the pair's second half contributes zero
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int f2 = (4 * g4 + q) * TP2 + 16 + j;
                T_d1[f2] = 0.f;
                T_e1[f2] = 0.f;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        const int rd = j * TP + 4 * g4;
        const f4 ad2 = *reinterpret_cast<const f4*>(T_d2 + rd);
        const f4 bh1 = *reinterpret_cast<const f4*>(T_h1 + rd);
        __builtin_amdgcn_wave_barrier();  // (the wave's LDS reads complete in order before its writes)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int fo = (4 * g4 + q) * TP + pr;
            T_e2[fo] = dc2[q];
            T_k1[fo] = f.hc1[q];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        const f4 ae2 = *reinterpret_cast<const f4*>(T_e2 + rd);
        const f4 bk1 = *reinterpret_cast<const f4*>(T_k1 + rd);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int fo = (4 * g4 + q) * TP + pr;
            T_h2[fo] = f.h2[q];
#pragma unroll
            for (int t = 0; t < (X1 ? NT - 1 : NT); t++) T_gz[t * 16 * TP + fo] = gz[t][q];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        const f4 bh2 = *reinterpret_cast<const f4*>(T_h2 + rd);
        f4 agz[NT];
#pragma unroll
        for (int t = 0; t < (X1 ? NT - 1 : NT); t++) agz[t] = *reinterpret_cast<const f4*>(T_gz + t * 16 * TP + rd);
#pragma unroll
        for (int s = 0; s < 4; s++) {
            gW2 = mfma4(ad2[s], bh1[s], gW2);
            gC2 = mfma4(ae2[s], bk1[s], gC2);
        }
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
            for (int t = 0; t < (X1 ? NT - 1 : NT); t++) gW3[t] = mfma4(agz[t][s], bh2[s], gW3[t]);
        if constexpr (X1) {
#pragma unroll
            for (int q = 0; q < 4; q++) gW3x[q] = fmaf(g16, f.h2[q], gW3x[q]);
        }
        if (pair_done) {
            // dW1 / dC1 over the pair's 32 rows on the bf16 MFMA: A = d1 (e1) of rows 8*g4..+7 of
            // hidden unit j as three exact bf16 terms, B = the int8 inputs of those rows; output
            // column j of tile q is input feature NQ*j + q
            float v[8];
            u4v dh, dm, dl, eh, em, el;
            const f4 d_lo = *reinterpret_cast<const f4*>(T_d1 + j * TP2 + 8 * g4);
            const f4 d_hi = *reinterpret_cast<const f4*>(T_d1 + j * TP2 + 8 * g4 + 4);
#pragma unroll
            for (int e = 0; e < 4; e++) v[e] = d_lo[e], v[4 + e] = d_hi[e];
            split3(v, dh, dm, dl);
            const f4 e_lo = *reinterpret_cast<const f4*>(T_e1 + j * TP2 + 8 * g4);
            const f4 e_hi = *reinterpret_cast<const f4*>(T_e1 + j * TP2 + 8 * g4 + 4);
#pragma unroll
            for (int e = 0; e < 4; e++) v[e] = e_lo[e], v[4 + e] = e_hi[e];
            split3(v, eh, em, el);
            // the NQ input bytes NQ*j .. NQ*j + NQ-1 of rows 8*g4 + r, a dword (4 tiles q) at a time
            constexpr int XW = (NQ + 3) / 4;
#pragma unroll
            for (int w = 0; w < XW; w++) {
                uint32_t xr8[8];
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const uint8_t* row = reinterpret_cast<const uint8_t*>(sX + (8 * g4 + r) * XPD) + NQ * j;
                    if (NQ == 1)
                        xr8[r] = row[0];
                    else if (NQ == 2)
                        xr8[r] = *reinterpret_cast<const uint16_t*>(row);
                    else
                        xr8[r] = reinterpret_cast<const uint32_t*>(row)[w];
                }
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    const int q = 4 * w + qq;
                    if (q >= NQ) break;
                    u4v xb;
#pragma unroll
                    for (int d = 0; d < 4; d++)
                        xb[d] = pack_i8((int)(int8_t)(xr8[2 * d] >> (8 * qq)), (int)(int8_t)(xr8[2 * d + 1] >> (8 * qq)));
                    gW1[q] = mfma_bf16(dh, xb, gW1[q]);
                    gW1[q] = mfma_bf16(dm, xb, gW1[q]);
                    gW1[q] = mfma_bf16(dl, xb, gW1[q]);
                    gC1[q] = mfma_bf16(eh, xb, gC1[q]);
                    gC1[q] = mfma_bf16(em, xb, gC1[q]);
                    gC1[q] = mfma_bf16(el, xb, gC1[q]);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    };

    // lane (j, g4) loads dwords 8s + 2*g4 + {0, 1} of row r (its bf16 B fragment of k-step s) and
    // row r's scalars (register prefetch: issued before the current tile is processed).
    // The rollout arrays are read as raw buffers whose base is a wave-uniform first row r0 (the
    // descriptors are built on the scalar unit): a lane's load is a 32-bit offset (r - r0) * row
    // bytes, with no 64-bit address arithmetic per row, and rows at or past R read 0.
    uint32_t pre[S1][2];
    int pre_act = 0;
    float pre_olp = 0.f, pre_G = 0.f;
    const int st_rb = (OWNROWS ? p.owner_C : (int)p.rrs) * p.stride;  // bytes between rows
    const int ac_rb = (int)p.rrs, lp_rb = 4 * (int)p.rrs, rt_rb = 4 * p.ret_ld;
    const int8_t* st_base =
        OWNROWS ? p.states + (size_t)own_c * p.stride : p.states + (size_t)u * (size_t)p.rus * p.stride;
    const int8_t* ac_base = p.actions + (size_t)u * (size_t)p.rus;
    const float* lp_base = p.old_lp + (size_t)u * (size_t)p.rus;
    const float* rt_base = p.ret + grp;
    struct RowBufs {
        __amdgpu_buffer_rsrc_t st, ac, lp, rt;
    };
    // rows per descriptor before its byte count passes 2^31 - 1 (32-bit scalar compares in the loop)
    const int lim_st = 0x7fffffff / st_rb, lim_lp = 0x7fffffff / max(lp_rb, rt_rb);
    auto row_bufs = [&](int r0) {  // r0 wave-uniform
        const int nrow = max(R - r0, 0);
        auto mk = [&](const void* base, int step, int lim) {
            const int n = nrow > lim ? 0x7fffffff : nrow * step;
            return __builtin_amdgcn_make_buffer_rsrc(
                const_cast<void*>(reinterpret_cast<const void*>(reinterpret_cast<const int8_t*>(base) +
                                                                (long long)r0 * step)),
                0, n, 0x00020000);
        };
        RowBufs b;
        b.st = mk(st_base, st_rb, lim_st);
        b.ac = mk(ac_base, ac_rb, lim_lp);
        b.lp = mk(lp_base, lp_rb, lim_lp);
        b.rt = mk(rt_base, rt_rb, lim_lp);
        return b;
    };
    int ccol[S1][2];  // this lane's dword columns of a row (clamped: the bytes past the row meet zero weights)
#pragma unroll
    for (int s = 0; s < S1; s++)
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int cc = 8 * s + 2 * g4 + h;
            ccol[s][h] = 4 * (cc < stride4 ? cc : stride4 - 1);
        }
    auto prefetch_rel = [&](const RowBufs& b, uint32_t rel) {  // row r0 + rel of b
#pragma unroll
        for (int s = 0; s < S1; s++)
#pragma unroll
            for (int h = 0; h < 2; h++)
                pre[s][h] = __builtin_amdgcn_raw_buffer_load_b32(b.st, (int)(__umul24(rel, st_rb) + ccol[s][h]), 0, 0);
        pre_act = (int8_t)__builtin_amdgcn_raw_buffer_load_b8(b.ac, (int)__umul24(rel, ac_rb), 0, 0);
        pre_olp = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(b.lp, (int)__umul24(rel, lp_rb), 0, 0));
        pre_G = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(b.rt, (int)__umul24(rel, rt_rb), 0, 0));
    };

    if constexpr (MODE == kKeyFwd || MODE == kKeyBack) {
        // ---- keyed rows, the passes over one group's distinct rows in rank order (16 ranks per
        //      tile, a contiguous range of tiles per wave). Fwd: the forward values of every rank.
        //      Back: the ranks' summed loss derivatives (k_key_scan's block sums, added in block
        //      order) through one backward pass per rank, exactly as the common row's virtual tile
        //      (the backward is linear in them)
        constexpr int KA = 16 * NT + 1, KF = 16 * NT + 4;
        const bool keyed = p.key_n[grp] >= 0 && p.key_flag[grp] == 0;
        const int n = keyed ? p.key_n[grp] : 0;
        const int tiles = (n + 15) / 16;
        const int wpg = p.blocks_per_group * L::WPB;
        const int tpw = (tiles + wpg - 1) / wpg;
        const int st0 = (blk * L::WPB + wave) * tpw, st1 = min(st0 + tpw, tiles);
        const size_t gr = (size_t)grp * kKeyMaxRanks;
        const double fx_lp = -(double)p.inv_R / kKeyFx, fx_v = (double)p.inv_R / kKeyFx;
        int otile = 0;
        for (int tile = st0; tile < st1; tile++) {
            const int rank = 16 * tile + j;
            const bool occ = rank < n;
            const uint32_t kw = occ ? p.key_sorted[gr + rank] : 0u;
            uint32_t xr[S1][2];
#pragma unroll
            for (int s = 0; s < S1; s++) xr[s][0] = xr[s][1] = 0u;
            xr[0][0] = g4 == 0 ? kw : 0u;  // a stride-4 row is dword 0 of k-step 0
            if constexpr (MODE == kKeyFwd) {
                Fwd f;
                forward(xr, f);
                const float ent_row = ent_of(f);  // (a cross-lane sum: outside the branches)
                if (occ) {
                    float* dst = p.key_fwd + (gr + rank) * KF;
#pragma unroll
                    for (int t = 0; t < NT; t++)
#pragma unroll
                        for (int q = 0; q < 4; q++) dst[16 * t + 4 * g4 + q] = f.cl[t][q];
                    if (g4 == 0) {
                        dst[16 * NT] = f.V;
                        dst[16 * NT + 1] = ent_row;
                    }
                }
            } else {
                long long acc[NT][4], accv = 0;
                uint32_t cnt = 0;
#pragma unroll
                for (int t = 0; t < NT; t++) acc[t][0] = acc[t][1] = acc[t][2] = acc[t][3] = 0;
                if (occ) {
                    for (int b = 0; b < p.key_nbs; b++) {
                        const size_t pr = ((size_t)grp * p.key_nbs + b) * kKeyMaxRanks + rank;
                        const long long* ac = p.key_part + pr * KA;
#pragma unroll
                        for (int t = 0; t < NT; t++)
#pragma unroll
                            for (int q = 0; q < 4; q++)
                                if (16 * t + 4 * g4 + q < A) acc[t][q] += ac[16 * t + 4 * g4 + q];
                        accv += ac[16 * NT];
                        cnt += p.key_pcnt[pr];
                    }
                }
                float vsum[NT][4];
#pragma unroll
                for (int t = 0; t < NT; t++)
#pragma unroll
                    for (int q = 0; q < 4; q++) vsum[t][q] = (float)((double)acc[t][q] * fx_lp);
                const float gv = (float)((double)accv * fx_v);
                const float gh = -0.01f * p.inv_R * (float)cnt;
                const int half = otile & 1;
                tile_step(BoolC<true>{}, xr, 0, 0.f, 0.f, true, half, half == 1, vsum, gh, gv);
                otile++;
            }
        }
        if constexpr (MODE == kKeyFwd) {
            return;
        } else {
            if (otile & 1) {  // the last pair's second half: a tile of zero derivatives
                uint32_t xr[S1][2];
#pragma unroll
                for (int s = 0; s < S1; s++) xr[s][0] = xr[s][1] = 0u;
                tile_step(BoolC<true>{}, xr, 0, 0.f, 0.f, true, 1, true, zero_vs, 0.f, 0.f);
            }
            if (keyed && blk == 0 && wave == 0 && lane == 0) {  // the scan blocks' loss sums, in block order
                for (int b = 0; b < p.key_nbs; b++) {
                    const float* ls = p.key_ploss + ((size_t)grp * p.key_nbs + b) * 4;
                    l_min += ls[0];
                    l_mse += ls[1];
                    l_ent += ls[2];
                }
            }
        }
    } else if constexpr (MODE == kPlain) {
        // rows past the end read zeros (row_bufs): their loss weight is 0, so every derivative of
        // theirs is exactly 0 (all inputs finite)
        if (tile0 < tile_end) prefetch_rel(row_bufs(16 * tile0), (uint32_t)j);
        for (int tile = tile0; tile < tile_end; tile++) {
            const int half = (tile - tile0) & 1;  // position in the tile pair of the dW1 step
            uint32_t xr[S1][2];
#pragma unroll
            for (int s = 0; s < S1; s++) xr[s][0] = pre[s][0], xr[s][1] = pre[s][1];
            const bool valid = tile * 16 + j < R;
            const int act = pre_act;
            const float olp = pre_olp, G = pre_G;
            if (tile + 1 < tile_end) prefetch_rel(row_bufs(16 * (tile + 1)), (uint32_t)j);
            tile_step(BoolC<false>{}, xr, act, olp, G, valid, half, half == 1 || tile + 1 == tile_end, zero_vs, 0.f,
                      0.f);
        }
    } else if constexpr (MODE == kMaskRow) {
        // ---- the rows the group's own-row mask lists (k_own_scan: bit r of word w = row 32w + r is
        //      the owner's row, or a common row whose term the fixed-point sums could not hold), in
        //      16-row tiles; this wave's chunk is a contiguous range of mask words. The common rows'
        //      summed derivatives (k_own_common) run through one virtual tile, on wave 0 of block 0.
        const int wpc = (p.own_words + p.n_chunks - 1) / p.n_chunks;
        const int w0 = min(chunk * wpc, p.own_words), w1 = min(w0 + CPW * wpc, p.own_words);
        const int rb = 32 * w0;
        int32_t* list = reinterpret_cast<int32_t*>(sCm);
        const uint32_t* mask = p.own_mask + (size_t)grp * p.own_words;
        const RowBufs wb = row_bufs(rb);
        int n_list = 0, otile = 0;
        auto list_tiles = [&](int cnt) {
            auto pf = [&](int t0) { prefetch_rel(wb, (uint32_t)(list[t0 + (t0 + j < cnt ? j : 0)] - rb)); };
            pf(0);
            for (int t0 = 0; t0 < cnt; t0 += 16) {
                uint32_t xr[S1][2];
#pragma unroll
                for (int s = 0; s < S1; s++) xr[s][0] = pre[s][0], xr[s][1] = pre[s][1];
                const int act = pre_act;
                const float olp = pre_olp, G = pre_G;
                const bool valid = t0 + j < cnt;
                if (t0 + 16 < cnt) pf(t0 + 16);
                const int half = otile & 1;
                tile_step(BoolC<false>{}, xr, act, olp, G, valid, half, half == 1, zero_vs, 0.f, 0.f);
                otile++;
            }
        };
        for (int wbase = w0; wbase < w1; wbase += 32) {
            // 32 mask words (1024 rows) per step: lane k < 32 expands word wbase + k into its rows, at
            // its exclusive prefix count of listed rows (rows stay in increasing order)
            const int w = wbase + lane;
            uint32_t m = (lane < 32 && w < w1) ? mask[w] : 0u;
            const int c = __popc(m);
            int incl = c;
#pragma unroll
            for (int d = 1; d < 32; d <<= 1) {
                const int v = __shfl_up(incl, d);
                if (lane >= d) incl += v;
            }
            const int total = __shfl(incl, 31);
            int pos = n_list + incl - c;
            while (m) {
                list[pos++] = 32 * w + __ffs(m) - 1;
                m &= m - 1;
            }
            n_list += total;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int full = n_list & ~15;
            if (full > 0) list_tiles(full);
            const int rest = n_list - full;
            const int mv = lane < rest ? list[full + lane] : 0;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < rest) list[lane] = mv;
            n_list = rest;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (n_list > 0) list_tiles(n_list);
        if (blk == 0 && wave == 0) {
            // the common rows of the whole group: column 0 of the virtual tile carries their summed
            // derivatives (k_own_common: per action, then sum of V - G, count, loss sums)
            const float* cs = p.own_csum + (size_t)grp * (16 * NT + 8);
            uint32_t txr[S1][2];
            const uint32_t* crow = reinterpret_cast<const uint32_t*>(p.common);
#pragma unroll
            for (int s = 0; s < S1; s++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int cc = 8 * s + 2 * g4 + h;
                    txr[s][h] = crow[cc < stride4 ? cc : stride4 - 1];
                }
            float vsum[NT][4];
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int q = 0; q < 4; q++) vsum[t][q] = j == 0 ? cs[16 * t + 4 * g4 + q] : 0.f;
            const float gv = cs[16 * NT], cnt = cs[16 * NT + 1];
            tile_step(BoolC<true>{}, txr, 0, 0.f, 0.f, true, otile & 1, true, vsum,
                      j == 0 ? -0.01f * p.inv_R * cnt : 0.f, j == 0 ? gv : 0.f);
            if (lane == 0) {
                l_min += cs[16 * NT + 2];
                l_mse += cs[16 * NT + 3];
                l_ent += cs[16 * NT + 4];
            }
        } else if (otile & 1) {  // the last pair's second half: a tile of zero derivatives
            uint32_t xr[S1][2];
#pragma unroll
            for (int s = 0; s < S1; s++) xr[s][0] = xr[s][1] = 0u;
            tile_step(BoolC<true>{}, xr, 0, 0.f, 0.f, true, 1, true, zero_vs, 0.f, 0.f);
        }
    } else if constexpr (L::CM) {
    if (tile0 < tile_end) {
        // ---- rows equal to the common row (acceptor rows of cores the agent does not own) share
        //      one forward pass: the wave scans its rows one per lane, accumulates their loss
        //      derivatives by action, and lists the other rows for the MFMA tiles; the summed
        //      derivatives then run through the common row's backward once (virtual tile)
        const int rb = tile0 * 16, re = min(tile_end * 16, R);
        int32_t* list = reinterpret_cast<int32_t*>(sCm + 16 * NT + 4);
        uint32_t txr[S1][2];
        const uint32_t* crow = reinterpret_cast<const uint32_t*>(p.common);
#pragma unroll
        for (int s = 0; s < S1; s++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int cc = 8 * s + 2 * g4 + h;
                txr[s][h] = crow[cc < stride4 ? cc : stride4 - 1];
            }
        constexpr int LPR = S1 <= 2 ? 4 : (S1 <= 4 ? 8 : 16);
        CommonScan<LPR> cs;
        if constexpr (MODE == kCommonRow) cs.init(crow, stride4, lane);
        {
            uint32_t xw[S1][2];
#pragma unroll
            for (int s = 0; s < S1; s++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int cc = 8 * s + 2 * g4 + h;
                    xw[s][h] = cc < stride4 ? txr[s][h] : 0u;
                }
            Fwd f;
            forward(xw, f);
            const float ent_row = ent_of(f);
            if (j == 0) {
#pragma unroll
                for (int t = 0; t < NT; t++)
#pragma unroll
                    for (int q = 0; q < 4; q++) sCm[16 * t + 4 * g4 + q] = f.cl[t][q];
                if (g4 == 0) {
                    sCm[16 * NT] = f.V;
                    sCm[16 * NT + 1] = ent_row;
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const float Vc = sCm[16 * NT], ent_c = sCm[16 * NT + 1];
        // the wave's sums of d min(surr)/d ratio * ratio per action over its common rows: int64
        // fixed point (2^-28) with LDS atomics, so the order of the adds does not matter; a row
        // whose term could overflow them is listed for the tiles instead
        constexpr int SEG = seg_rows<MODE>();
        long long* vacc = reinterpret_cast<long long*>(list + SEG + 64);
        if (lane < 16 * NT) vacc[lane] = 0;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float qbound = 34359738368.f / (float)max(re - rb, 1);  // |q| * 2^28 * rows < 2^63
        float sgv = 0.f, sl_min = 0.f, sl_mse = 0.f, sl_ent = 0.f;
        int scnt = 0;
        const uint64_t below = (1ull << lane) - 1ull;
        int n_list = 0, otile = 0;
        // scan registers, kScanDepth 64-row steps in flight: the rows' chunks (cooperative 16-byte
        // loads) and row r0 + lane's scalars
        constexpr int PF = MODE == kOwnerRow ? kScanDepthOwn : kScanDepth;
        u4a sc[MODE == kCommonRow ? PF : 1][MODE == kCommonRow ? LPR : 1];
        int s_act[PF];
        int8_t s_own[PF];
        float s_olp[PF], s_G[PF];
        // the wave's rows as raw buffers from row rb (32-bit per-lane offsets)
        const RowBufs wb = row_bufs(rb);
        const __amdgpu_buffer_rsrc_t ob =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(MODE == kOwnerRow ? p.owner + (size_t)rb * p.owner_C + own_c
                                                                                     : p.actions),
                                              0, MODE == kOwnerRow ? (int)((re - rb) * p.owner_C) : 0, 0x00020000);
        auto load_slot = [&](int k, int r0, int lim) {
            if constexpr (MODE == kCommonRow)
                cs.load_into(sc[k], [&](int q) { return row_src(r0 + q < lim ? r0 + q : rb); }, lane);
            const int r = r0 + lane;
            const uint32_t rel = (uint32_t)((r < lim ? r : rb) - rb);
            if constexpr (MODE == kOwnerRow)
                s_own[k] = (int8_t)__builtin_amdgcn_raw_buffer_load_b8(ob, (int)__umul24(rel, p.owner_C), 0, 0);
            s_act[k] = (int8_t)__builtin_amdgcn_raw_buffer_load_b8(wb.ac, (int)__umul24(rel, ac_rb), 0, 0);
            s_olp[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wb.lp, (int)__umul24(rel, lp_rb), 0, 0));
            s_G[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wb.rt, (int)__umul24(rel, rt_rb), 0, 0));
        };
        // the listed rows t0 .. t0 + 16*n - 1 (the last tile may be partial: cnt rows in all) in
        // 16-row tiles, the next tile's rows prefetched
        auto owner_tiles = [&](int cnt) {
            auto pf = [&](int t0) { prefetch_rel(wb, (uint32_t)(list[t0 + (t0 + j < cnt ? j : 0)] - rb)); };
            pf(0);
            for (int t0 = 0; t0 < cnt; t0 += 16) {
                uint32_t xr[S1][2];
#pragma unroll
                for (int s = 0; s < S1; s++) xr[s][0] = pre[s][0], xr[s][1] = pre[s][1];
                const int act = pre_act;
                const float olp = pre_olp, G = pre_G;
                const bool valid = t0 + j < cnt;
                if (t0 + 16 < cnt) pf(t0 + 16);
                const int half = otile & 1;
                tile_step(BoolC<false>{}, xr, act, olp, G, valid, half, half == 1, zero_vs, 0.f, 0.f);
                otile++;
            }
        };
        for (int seg = rb; seg < re; seg += SEG) {
            const int seg_end = min(seg + SEG, re);
#pragma unroll
            for (int k = 0; k < PF; k++)
                if (seg + 64 * k < seg_end) load_slot(k, seg + 64 * k, seg_end);
            for (int rs0 = seg; rs0 < seg_end; rs0 += 64 * PF) {
#pragma unroll
                for (int k = 0; k < PF; k++) {
                    const int r0 = rs0 + 64 * k;
                    if (r0 >= seg_end) break;
                    const int r = r0 + lane;
                    const bool in = r < seg_end;
                    bool common;
                    if constexpr (MODE == kOwnerRow)
                        common = s_own[k] != own_me && in;
                    else
                        common = cs.common_of(sc[k], lane) && in;
                    const int act = s_act[k];
                    const float olp = s_olp[k], G = s_G[k];
                    if (r0 + 64 * PF < seg_end) load_slot(k, r0 + 64 * PF, seg_end);
                    float qd = 0.f, sur1 = 0.f, sur2 = 0.f;
                    if (common) {
                        // the tile path's per-row derivatives with the common row's forward values
                        const float lp = (unsigned)act < (unsigned)A ? sCm[act] : 0.f;
                        const float ratio = fast_exp(lp - olp);
                        const float adv = G - Vc;
                        sur1 = ratio * adv;
                        const float rc = fminf(fmaxf(ratio, 1.f - p.eps_clip), 1.f + p.eps_clip);
                        sur2 = rc * adv;
                        const float inr = (ratio >= 1.f - p.eps_clip && ratio <= 1.f + p.eps_clip) ? 1.f : 0.f;
                        const float dmin =
                            sur1 < sur2 ? adv : (sur2 < sur1 ? adv * inr : 0.5f * adv + 0.5f * adv * inr);
                        qd = dmin * ratio;
                        common = fabsf(qd) <= qbound;  // NaN or huge: the tile path
                    }
                    if (common) {
                        if ((unsigned)act < (unsigned)A)
                            atomicAdd(reinterpret_cast<unsigned long long*>(vacc + act),
                                      (unsigned long long)__float2ll_rn(qd * 268435456.f));
                        sgv += (Vc - G) * p.inv_R;
                        scnt++;
                        sl_min += -fminf(sur1, sur2);
                        sl_mse += (Vc - G) * (Vc - G);
                        sl_ent += ent_c;
                    }
                    const bool other = in && !common;
                    const uint64_t m = __ballot(other);
#ifdef MS_GRAD_PROBE
                    probe_listed += __popcll(m);
#endif
                    if (other) list[n_list + __popcll(m & below)] = r;
                    n_list += __popcll(m);
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int full = n_list & ~15;
            if (full > 0) owner_tiles(full);
            // the rest (< 16 rows) moves to the front of the list
            const int rest = n_list - full;
            const int mv = lane < rest ? list[full + lane] : 0;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < rest) list[lane] = mv;
            n_list = rest;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (n_list > 0) owner_tiles(n_list);
#ifdef MS_GRAD_PROBE
        probe_t1 = __builtin_amdgcn_s_memrealtime();
#endif
        // the virtual tile: column 0 carries the common rows' summed derivatives
        // wave totals per action (lane k sums action k's 64 entries in lane order), then column 0
        // of the virtual tile: lane (0, g4) takes actions 16t + 4*g4 + q
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const double fx_lp = -(double)p.inv_R / 268435456.0;
        float vsum[NT][4];
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) vsum[t][q] = j == 0 ? (float)((double)vacc[16 * t + 4 * g4 + q] * fx_lp) : 0.f;
        const float gv_tot = xsum16(xsum4g(sgv));
        const float cnt_tot = (float)(int)xsum16(xsum4g((float)scnt));
        tile_step(BoolC<true>{}, txr, 0, 0.f, 0.f, true, otile & 1, true, vsum, j == 0 ? -0.01f * p.inv_R * cnt_tot : 0.f,
                  j == 0 ? gv_tot : 0.f);
        // the common rows' loss terms join lane group 0's sums
        const float m_tot = xsum16(xsum4g(sl_min)), q_tot = xsum16(xsum4g(sl_mse)), e_tot = xsum16(xsum4g(sl_ent));
        if (lane == 0) {
            l_min += m_tot;
            l_mse += q_tot;
            l_ent += e_tot;
        }
    }
    }

    // ---- the block's partial gradient: the 4 waves' vectors summed in LDS in wave order
    //      (deterministic), then one coalesced store per block
    const POff o = poff(D, A);
    auto write_partial = [&](auto&& put) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int f = 4 * g4 + q;  // C row (output feature) held in register q
#pragma unroll
            for (int qq = 0; qq < NQ; qq++) {
                const int d = NQ * j + qq;
                if (d < D) {
                    put(o.w1 + f * D + d, gW1[qq][q]);
                    put(o.cw1 + f * D + d, gC1[qq][q]);
                } else if (d == D) {  // the ones column: layer-1 bias gradients
                    put(o.b1 + f, gW1[qq][q]);
                    put(o.cb1 + f, gC1[qq][q]);
                }
            }
            put(o.w2 + f * 16 + j, gW2[q]);
            put(o.cw2 + f * 16 + j, gC2[q]);
#pragma unroll
            for (int t = 0; t < (X1 ? NT - 1 : NT); t++) {
                const int a = 16 * t + f;
                if (a < A) put(o.w3 + a * 16 + j, gW3[t][q]);
            }
            if constexpr (X1) {  // row 16 (NT - 1) of dW3: unit f, summed over the 16 row lanes
                const float v3 = xsum16(gW3x[q]);
                if (j == 0) put(o.w3 + 16 * (NT - 1) * 16 + f, v3);
            }
            float v;
            v = xsum16(db2[q]);
            if (j == 0) put(o.b2 + f, v);
            v = xsum16(cdb2[q]);
            if (j == 0) put(o.cb2 + f, v);
            v = xsum16(gC3[q]);
            if (j == 0) put(o.cw3 + f, v);
#pragma unroll
            for (int t = 0; t < NT; t++) {
                v = xsum16(db3[t][q]);
                if (j == 0 && 16 * t + f < A) put(o.b3 + 16 * t + f, v);
            }
        }
        float v = xsum16(cdb3);
        if (lane == 0) put(o.cb3, v);
        v = xsum16(l_min);
        if (lane == 0) put(o.loss + 0, v * p.inv_R);
        v = xsum16(l_mse);
        if (lane == 0) put(o.loss + 1, v * p.inv_R);
        v = xsum16(l_ent);
        if (lane == 0) put(o.loss + 2, v * p.inv_R);
    };
    __syncthreads();  // every wave is done with the weights and its transposes
    float* acc = sm;
    for (int wv = 0; wv < L::WPB; wv++) {
        if (wave == wv) {
            auto put = [&](int i, float x) {
                if (wv == 0)
                    acc[i] = x;
                else
                    acc[i] += x;
            };
            write_partial(put);
        }
        __syncthreads();
    }
    float* outp = p.partials + ((size_t)grp * p.part_rows + p.part_off + blk) * p.P;
    for (int i = tid; i < p.P; i += NTH) outp[i] = acc[i];
#ifdef MS_GRAD_PROBE
    if constexpr (L::CM) {
        const int wi = blockIdx.x * L::WPB + wave;
        if (lane == 0 && wi < kGradProbeWaves) {
            g_grad_probe[wi][0] = probe_t0;
            g_grad_probe[wi][1] = probe_t1;
            g_grad_probe[wi][2] = __builtin_amdgcn_s_memrealtime();
            g_grad_probe[wi][3] = probe_listed | ((unsigned long long)grp << 32);
        }
    }
#endif
}

// ---- compact acceptor rows of many groups (the divided acceptors of cfg4: 256 nets, each on its own
//      1.6 M rows, of which ~5 % are its own rows). PPOmodules.py:127-174 per group; Agent.py:167-212:
//      an acceptor row is its core's owner row when the agent owns the core, else the constant
//      common (foreign) row, whose forward is the same for every such row of a group.
// k_own_scan: one pass over the rows for 64 groups at a time, lane = group (the [R][U] rollout rows
// of 64 consecutive units are 64 contiguous bytes / floats, so every load is one coalesced segment;
// the per-group scans of the tile kernel read 1-4 bytes of each row's line). For a common row the
// lane adds the tile path's d min(surr)/d ratio * ratio to its group's int64 fixed-point sum of the
// row's action (LDS, [A][64]: no two lanes share an address), and (V - G)/R, the count and the loss
// terms to its registers; every other row (the owner's, or a term beyond own_qbound) gets its bit in
// the group's mask for the tiles. Block = 4 waves on consecutive kOwnScanRows-row chunks of the same
// 64 groups; the block's sums go to own_part, each wave's floats to own_wpart (fixed order later).
__global__ void __launch_bounds__(256) k_own_scan(PpoArgs p) {
    extern __shared__ __align__(16) long long own_sh[];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int A = p.A, KA = 16 * ((A + 15) / 16);
    const int g = blockIdx.y * 64 + lane;
    const bool gok = g < p.G;
    long long* sums = own_sh;                                   // [A][64]
    float* cl = reinterpret_cast<float*>(own_sh + A * 64);      // [A][64]
    float* vt = cl + A * 64;                                    // [2][64]: V, entropy of the common row
    for (int i = tid; i < A * 64; i += 256) {
        const int a = i >> 6, gg = blockIdx.y * 64 + (i & 63);
        sums[i] = 0;
        cl[i] = gg < p.G ? p.own_cfwd[(size_t)gg * (KA + 4) + a] : 0.f;
    }
    if (tid < 128) {
        const int gg = blockIdx.y * 64 + (tid & 63);
        vt[tid] = gg < p.G ? p.own_cfwd[(size_t)gg * (KA + 4) + KA + (tid >> 6)] : 0.f;
    }
    __syncthreads();
    const int u = gok ? p.unit_of_group[g] : 0;
    const int own_c = u % p.owner_C;
    const int own_me = u / p.owner_C + 1;
    const float Vc = vt[lane], ent_c = vt[64 + lane];
    const int wc = blockIdx.x * 4 + wave;  // this wave's chunk of rows
    const long long r0 = (long long)wc * kOwnScanRows;
    const int nrow = (int)max(0LL, min((long long)kOwnScanRows, p.R - r0));
    // the chunk's rows as raw buffers from row r0: the wave-uniform row offset goes in soffset, the
    // lane's column in voffset (no per-row address arithmetic)
    auto mk = [&](const void* base, long long step) {
        return __builtin_amdgcn_make_buffer_rsrc(
            const_cast<void*>(reinterpret_cast<const void*>(reinterpret_cast<const int8_t*>(base) + r0 * step)), 0,
            (int)(nrow * step), 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t b_ac = mk(p.actions, p.rrs), b_lp = mk(p.old_lp, 4 * p.rrs),
                                 b_rt = mk(p.ret, 4LL * p.ret_ld), b_ow = mk(p.owner, p.owner_C);
    const int c_ac = (int)(u * p.rus), c_lp = 4 * c_ac, c_rt = 4 * g, c_ow = own_c;
    const int s_ac = (int)p.rrs, s_lp = 4 * (int)p.rrs, s_rt = 4 * p.ret_ld, s_ow = p.owner_C;
    const float qb = p.own_qbound, eps_lo = 1.f - p.eps_clip, eps_hi = 1.f + p.eps_clip;
    float sgv = 0.f, sl_min = 0.f, sl_mse = 0.f, sl_ent = 0.f;
    int scnt = 0;
    uint32_t* mrow = p.own_mask + (size_t)g * p.own_words + (size_t)r0 / 32;
    constexpr int U8 = 8;  // rows per batch of loads
    for (int w = 0; 32 * w < nrow; w++) {
        uint32_t bits = 0;
#pragma unroll
        for (int k8 = 0; k8 < 32; k8 += U8) {
            int act[U8], ow[U8];
            float olp[U8], G[U8];
#pragma unroll
            for (int k = 0; k < U8; k++) {
                // rows past the chunk load the last row again (a wave-uniform clamp: soffset is not
                // part of the buffer's range check); the `in` test below drops them
                const int rr = min(32 * w + k8 + k, nrow - 1);
                act[k] = (int8_t)__builtin_amdgcn_raw_buffer_load_b8(b_ac, c_ac, rr * s_ac, 0);
                olp[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(b_lp, c_lp, rr * s_lp, 0));
                G[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(b_rt, c_rt, rr * s_rt, 0));
                ow[k] = (int8_t)__builtin_amdgcn_raw_buffer_load_b8(b_ow, c_ow, rr * s_ow, 0);
            }
#pragma unroll
            for (int k = 0; k < U8; k++) {
                const int rr = 32 * w + k8 + k;
                const bool in = gok && rr < nrow;
                bool common = in && ow[k] != own_me;
                float qd = 0.f, sur1 = 0.f, sur2 = 0.f;
                if (common) {
                    // the tile path's per-row derivatives with the common row's forward values
                    const float lp = (unsigned)act[k] < (unsigned)A ? cl[act[k] * 64 + lane] : 0.f;
                    const float ratio = fast_exp(lp - olp[k]);
                    const float adv = G[k] - Vc;
                    sur1 = ratio * adv;
                    const float rc = fminf(fmaxf(ratio, eps_lo), eps_hi);
                    sur2 = rc * adv;
                    const float inr = (ratio >= eps_lo && ratio <= eps_hi) ? 1.f : 0.f;
                    const float dmin = sur1 < sur2 ? adv : (sur2 < sur1 ? adv * inr : 0.5f * adv + 0.5f * adv * inr);
                    qd = dmin * ratio;
                    common = fabsf(qd) <= qb;  // NaN or huge: the tile path
                }
                if (common) {
                    if ((unsigned)act[k] < (unsigned)A)
                        atomicAdd(reinterpret_cast<unsigned long long*>(sums + act[k] * 64 + lane),
                                  (unsigned long long)__float2ll_rn(qd * 268435456.f));
                    sgv += (Vc - G[k]) * p.inv_R;
                    scnt++;
                    sl_min += -fminf(sur1, sur2);
                    sl_mse += (Vc - G[k]) * (Vc - G[k]);
                    sl_ent += ent_c;
                }
                if (in && !common) bits |= 1u << (k8 + k);
            }
        }
        if (gok) mrow[w] = bits;
    }
    if (gok) {
        float* wp = p.own_wpart + ((size_t)g * 4 * p.own_nb + wc) * 8;
        wp[0] = sgv;
        wp[1] = (float)scnt;
        wp[2] = sl_min;
        wp[3] = sl_mse;
        wp[4] = sl_ent;
    }
    __syncthreads();
    for (int i = tid; i < A * 64; i += 256) {
        const int a = i >> 6, gg = blockIdx.y * 64 + (i & 63);
        if (gg < p.G) p.own_part[((size_t)gg * p.own_nb + blockIdx.x) * A + a] = sums[i];
    }
}

// k_own_common: per group, the scan blocks' int64 sums (exact, order-free) and the scan waves' float
// sums (a fixed order: thread t takes waves t, t + 256, ..., then a fixed tree) -> own_csum:
// [16*NT] d loss / d log p of the common rows per action (= -sum / R, column 0 of the virtual tile),
// then sum of (V - G)/R, the count, and the three loss sums.
__global__ void __launch_bounds__(256) k_own_common(PpoArgs p) {
    __shared__ long long ps[2][128];
    __shared__ float pf[5][256];
    const int g = blockIdx.x, tid = threadIdx.x, A = p.A, KA = 16 * ((A + 15) / 16);
    const int a = tid & 127, part = tid >> 7;  // actions a (< 128) over two halves of the blocks
    long long s = 0;
    if (a < A)
        for (int b = part; b < p.own_nb; b += 2) s += p.own_part[((size_t)g * p.own_nb + b) * A + a];
    ps[part][a] = s;
    float f[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int wv = tid; wv < 4 * p.own_nb; wv += 256) {
        const float* wp = p.own_wpart + ((size_t)g * 4 * p.own_nb + wv) * 8;
#pragma unroll
        for (int k = 0; k < 5; k++) f[k] += wp[k];
    }
#pragma unroll
    for (int k = 0; k < 5; k++) pf[k][tid] = f[k];
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (tid < h)
#pragma unroll
            for (int k = 0; k < 5; k++) pf[k][tid] += pf[k][tid + h];
        __syncthreads();
    }
    float* cs = p.own_csum + (size_t)g * (KA + 8);
    const double fx_lp = -(double)p.inv_R / 268435456.0;
    if (tid < KA) cs[tid] = tid < A ? (float)((double)(ps[0][tid] + ps[1][tid]) * fx_lp) : 0.f;
    if (tid < 5) cs[KA + tid] = pf[tid][0];
}

// Sum the blocks' partial vectors (fixed order: 4 interleaved row sets, then a fixed tree) and
// scatter into the .grad tensors. Block = 64 parameters x 4 row sets.
__global__ void __launch_bounds__(256) k_ppo_reduce(const float* __restrict__ partials, int G, int n_rows, int P,
                                                    int D, int A, GradOut go, const int32_t* key_n,
                                                    const int32_t* key_flag, int key_rows) {
    __shared__ float part[4][64];
    const int grp = blockIdx.y;
    const int n_used = (key_n && key_n[grp] >= 0 && key_flag[grp] == 0) ? key_rows : n_rows;  // keyed: no tile rows
    const int pi = threadIdx.x & 63, rs = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + pi;
    float s = 0.f;
    if (i < P) {
        const float* src = partials + (size_t)grp * n_rows * P + i;
        for (int c = rs; c < n_used; c += 4) s += src[(size_t)c * P];
    }
    part[rs][pi] = s;
    __syncthreads();
    if (rs != 0 || i >= P) return;
    s = (part[0][pi] + part[1][pi]) + (part[2][pi] + part[3][pi]);
    const POff o = poff(D, A);
    float* dst;
    int k, base;
    if (i < o.b1) { dst = go.w1; k = 16 * D; base = o.w1; }
    else if (i < o.w2) { dst = go.b1; k = 16; base = o.b1; }
    else if (i < o.b2) { dst = go.w2; k = 256; base = o.w2; }
    else if (i < o.w3) { dst = go.b2; k = 16; base = o.b2; }
    else if (i < o.b3) { dst = go.w3; k = 16 * A; base = o.w3; }
    else if (i < o.cw1) { dst = go.b3; k = A; base = o.b3; }
    else if (i < o.cb1) { dst = go.cw1; k = 16 * D; base = o.cw1; }
    else if (i < o.cw2) { dst = go.cb1; k = 16; base = o.cb1; }
    else if (i < o.cb2) { dst = go.cw2; k = 256; base = o.cw2; }
    else if (i < o.cw3) { dst = go.cb2; k = 16; base = o.cb2; }
    else if (i < o.cb3) { dst = go.cw3; k = 16; base = o.cw3; }
    else if (i < o.loss) { dst = go.cb3; k = 1; base = o.cb3; }
    else { dst = go.loss; k = 3; base = o.loss; }
    if (dst) dst[(size_t)grp * k + (i - base)] = s;
}

template <int NQ, int NT, int MODE>
static hipError_t launch_grad_cm(const PpoArgs& a, unsigned blocks_per_group, hipStream_t st) {
    using L = GradLds<NQ, NT, MODE>;
    const size_t lds = sizeof(float) * L::lds_floats;
    if (lds > 160 * 1024 || (size_t)a.P > (size_t)L::lds_floats) return hipErrorInvalidValue;  // partial in LDS
    PpoArgs b = a;
    b.blocks_per_group = (int)blocks_per_group;
#if MS_XCD_MAP
    const unsigned grid = (unsigned)a.G * ((blocks_per_group + 7) / 8 * 8);
#else
    const unsigned grid = (unsigned)a.G * blocks_per_group;
#endif
    hipLaunchKernelGGL((k_ppo_grad<NQ, NT, MODE>), dim3(grid), dim3(64 * L::WPB), lds, st, b);
    return hipGetLastError();
}

// ---- keyed rows (nets of <= 4 inputs on 4-byte rows, e.g. the price chooser PPOmodules.py:327-330:
//      a few hundred distinct rows among millions). A row's dense index packs its bytes + 8, 5 bits
//      each; a group with a byte outside [-8, 24) takes the tile path.
__device__ __forceinline__ bool key_index(uint32_t w, int D, uint32_t& idx) {
    bool ok = true;
    idx = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        if (b < D) {
            const int v = (int)(int8_t)(w >> (8 * b)) + 8;
            ok &= (unsigned)v < 32u;
            idx |= (uint32_t)(v & 31) << (5 * b);
        }
    }
    return ok;
}

// the keyed passes' marks and flags to zero. A kernel, not hipMemsetAsync: in a replayed HIP graph the
// captured memset of the marks was not reliably complete before k_key_gather read them (marks left from
// the previous replay added ranks of no rows, which changed the backward's tile sums in the last bits;
// the update-streams test caught it, profiles/r7k)
__global__ void __launch_bounds__(256) k_key_clear(uint4* mark, size_t n16, int32_t* flag, int G) {
    const size_t i0 = (size_t)blockIdx.x * 256 + threadIdx.x, step = (size_t)gridDim.x * 256;
    for (size_t i = i0; i < n16; i += step) mark[i] = make_uint4(0u, 0u, 0u, 0u);
    for (size_t i = i0; i < (size_t)G; i += step) flag[i] = 0;
}

// one pass over the rows: every group's (dense index, action, old log-prob, return) to contiguous
// per-group arrays (so the scan reads whole lines instead of one unit's bytes of [R][U] rows), and
// every row's dense index marked (a load first: the frequent rows' marks are set early; every writer
// of a mark writes the same byte). Thread = row, all groups.
__global__ void __launch_bounds__(256) k_key_gather(PpoArgs p) {
    const uint32_t kmask = p.D >= 4 ? 0xffffffffu : ((1u << (8 * p.D)) - 1u);
    constexpr int GB = 8;  // groups per batch: all their loads are issued before any store
    for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < p.R; r += (long long)gridDim.x * 256) {
        for (int g0 = 0; g0 < p.G; g0 += GB) {
            uint32_t w[GB], idx[GB];
            int8_t act[GB];
            float olp[GB], ret[GB];
            uint8_t mk[GB];
#pragma unroll
            for (int k = 0; k < GB; k++) {
                const int grp = min(g0 + k, p.G - 1);
                const int u = p.unit_of_group[grp];
                const size_t ri = ru_index(p, r, u);
                w[k] = *reinterpret_cast<const uint32_t*>(p.states + ri * p.stride) & kmask;
                act[k] = p.actions[ri];
                olp[k] = p.old_lp[ri];
                ret[k] = p.ret[(size_t)r * p.ret_ld + grp];
            }
#pragma unroll
            for (int k = 0; k < GB; k++) {
                const int grp = min(g0 + k, p.G - 1);
                if (!key_index(w[k], p.D, idx[k]))
                    __hip_atomic_store(p.key_flag + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                mk[k] = p.key_mark[(size_t)grp * kKeyDense + idx[k]];
            }
#pragma unroll
            for (int k = 0; k < GB; k++) {
                if (g0 + k >= p.G) break;
                const int grp = g0 + k;
                if (mk[k] == 0) p.key_mark[(size_t)grp * kKeyDense + idx[k]] = 1;
                const size_t c = (size_t)grp * p.R + r;
                p.key_idx[c] = idx[k];
                p.key_act[c] = act[k];
                p.key_olp[c] = olp[k];
                p.key_ret[c] = ret[k];
            }
        }
    }
}

// k_key_gather for [R][U] rollout rows (rus == 1, rrs == U, U <= 64): a wave stages 64 consecutive rows of
// one array at a time in its LDS with coalesced 16-byte loads (the rows are contiguous), then each lane
// (= row) picks its groups' units from there, so no load instruction strides across rows (the per-lane
// loads of k_key_gather touch one 128-byte line per lane). Same outputs as k_key_gather.
constexpr int kGatherWaves = 4;
__global__ void __launch_bounds__(64 * kGatherWaves) k_key_gather_rows(PpoArgs p) {
    extern __shared__ __align__(16) uint32_t s_stage[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int U = (int)p.rrs, G = p.G, RL = (int)p.ret_ld;
    const int pitch = (U > RL ? U : RL) + 1;  // dwords per staged row (+1: the lanes of one read hit distinct banks)
    uint32_t* st = s_stage + (size_t)wave * 64 * pitch;
    const uint32_t kmask = p.D >= 4 ? 0xffffffffu : ((1u << (8 * p.D)) - 1u);
    const long long n_chunks = (p.R + 63) >> 6;
    // 64 rows x n dwords of src (row r0 + k at src + (r0 + k) * n) -> st[k * pitch + col]; rows past R are not
    // read, and the last row only up to column `last` (an array may be a column window of a wider one)
    auto stage = [&](const uint32_t* src, long long r0, int n, int last) {
        const int rows = (int)min(64ll, p.R - r0);
        const int total = (rows - 1) * n + last;  // dwords
        const uint32_t* base = src + r0 * n;
        const uint32_t mag = n > 1 ? 0xffffffffu / (uint32_t)n + 1u : 0u;  // d / n = umulhi(d, mag) for d < 2^12
        for (int d0 = 4 * lane; d0 < total; d0 += 256) {
            uint32_t v[4];
            if (d0 + 3 < total && ((reinterpret_cast<uintptr_t>(base + d0) & 15) == 0)) {
                const uint4 q = *reinterpret_cast<const uint4*>(base + d0);
                v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++) v[i] = d0 + i < total ? base[d0 + i] : 0u;
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int d = d0 + i;
                if (d < total) {
                    const int row = n > 1 ? (int)__umulhi((uint32_t)d, mag) : d;
                    st[row * pitch + (d - row * n)] = v[i];
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto done = [&]() {  // the staged values are read before the next stage overwrites them
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    for (long long ch = (long long)blockIdx.x * kGatherWaves + wave; ch < n_chunks;
         ch += (long long)gridDim.x * kGatherWaves) {
        const long long r0 = ch << 6, r = r0 + lane;
        const bool in = r < p.R;
        // dense indices (and marks) from the state words
        stage(reinterpret_cast<const uint32_t*>(p.states), r0, U, U);
        for (int g = 0; g < G; g++) {
            const int u = p.unit_of_group[g];
            uint32_t idx;
            const bool ok = key_index(st[lane * pitch + u] & kmask, p.D, idx);
            if (in) {
                if (!ok) __hip_atomic_store(p.key_flag + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                uint8_t* mk = p.key_mark + (size_t)g * kKeyDense + idx;
                if (*mk == 0) *mk = 1;
                p.key_idx[(size_t)g * p.R + r] = idx;
            }
        }
        done();
        stage(reinterpret_cast<const uint32_t*>(p.old_lp), r0, U, U);
        for (int g = 0; g < G; g++)
            if (in) p.key_olp[(size_t)g * p.R + r] = __uint_as_float(st[lane * pitch + p.unit_of_group[g]]);
        done();
        // returns: p.ret may be a column window of a wider [R][ret_ld] array (a later draw's groups), so
        // the last row is read only up to column G (the window's end in memory)
        stage(reinterpret_cast<const uint32_t*>(p.ret), r0, RL, G);
        for (int g = 0; g < G; g++)
            if (in) p.key_ret[(size_t)g * p.R + r] = __uint_as_float(st[lane * pitch + g]);
        done();
        // actions: U bytes per row, staged as dwords (U % 4 == 0)
        stage(reinterpret_cast<const uint32_t*>(p.actions), r0, U >> 2, U >> 2);
        const uint8_t* sa = reinterpret_cast<const uint8_t*>(st);
        for (int g = 0; g < G; g++)
            if (in) p.key_act[(size_t)g * p.R + r] = (int8_t)sa[lane * pitch * 4 + p.unit_of_group[g]];
        done();
    }
}

// the row word of a dense index
__device__ __forceinline__ uint32_t key_word_of(uint32_t idx, int D) {
    uint32_t w = 0;
#pragma unroll
    for (int b = 0; b < 4; b++)
        if (b < D) w |= (uint32_t)(uint8_t)(int8_t)((int)((idx >> (5 * b)) & 31u) - 8) << (8 * b);
    return w;
}

// ranks = the occurring dense indices in ascending order (a block-wide scan per group), so every
// later pass runs in an order that depends only on the set of distinct rows: deterministic
__global__ void __launch_bounds__(1024) k_key_rank(PpoArgs p) {
    __shared__ int part[1024];
    const int grp = blockIdx.x, tid = threadIdx.x;
    if (p.key_flag[grp]) {
        if (tid == 0) p.key_n[grp] = -1;
        return;
    }
    constexpr int PER = kKeyDense / 1024;  // contiguous indices per thread
    const size_t o = (size_t)grp * kKeyDense + (size_t)tid * PER;
    const uint4* m4 = reinterpret_cast<const uint4*>(p.key_mark + o);
    int c = 0;
    for (int k = 0; k < PER / 16; k++) {
        const uint4 v = m4[k];
        c += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);  // marks are 0 or 1
    }
    part[tid] = c;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // inclusive scan
        const int x = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    const int n = part[1023];
    int rk = part[tid] - c;
    if (n <= kKeyMaxRanks) {
        for (int k = 0; k < PER / 16 && c > 0; k++) {
            const uint4 v = m4[k];
            if ((v.x | v.y | v.z | v.w) == 0u) continue;
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
            for (int b = 0; b < 16; b++) {
                if ((wv[b >> 2] >> (8 * (b & 3))) & 0xffu) {
                    const size_t d = o + 16 * k + b;
                    p.key_rank[d] = rk;
                    p.key_sorted[(size_t)grp * kKeyMaxRanks + rk] = key_word_of((uint32_t)(16 * k + b + tid * PER), p.D);
                    rk++;
                }
            }
        }
    }
    if (tid == 0) p.key_n[grp] = n <= kKeyMaxRanks ? n : -1;
}

// the row scan: every row of the group looks up its rank and forward values and adds
// d min(surr) / d ratio * ratio (at its action), V - G and 1 to its rank's int64 sums in LDS (the
// sums do not depend on the order of the adds); ranks in passes of key_cap; then the block's sums
// and loss terms go to its own slice of key_part / key_pcnt / key_ploss with plain stores
template <int NT>
__global__ void __launch_bounds__(1024) k_key_scan(PpoArgs p) {
    constexpr int KA = 16 * NT + 1, KF = 16 * NT + 4;
    extern __shared__ __align__(16) long long sacc[];  // [cap][KA], then uint32 cnt[cap]
    __shared__ float red[3][1024];
    const int grp = blockIdx.x % p.G, blk = blockIdx.x / p.G, tid = threadIdx.x;
    const int n = p.key_n[grp];
    if (n < 0) return;
    uint32_t* scnt = reinterpret_cast<uint32_t*>(sacc + (size_t)p.key_cap * KA);
    const long long r_lo = p.R * blk / p.key_nbs, r_hi = p.R * (blk + 1) / p.key_nbs;
    const size_t gd = (size_t)grp * kKeyDense, gr = (size_t)grp * kKeyMaxRanks, gc = (size_t)grp * p.R;
    const size_t pb = (size_t)grp * p.key_nbs + blk;
    const float fx = (float)kKeyFx;
    float l_min = 0.f, l_mse = 0.f, l_ent = 0.f;
    bool bad = false;
    constexpr int UN = 4;  // rows in flight per thread
    for (int lo = 0; lo < n; lo += p.key_cap) {
        const int hi = min(lo + p.key_cap, n), nr = hi - lo;
        for (int i = tid; i < nr * KA; i += 1024) sacc[i] = 0;
        for (int i = tid; i < nr; i += 1024) scnt[i] = 0u;
        __syncthreads();
        for (long long r0 = r_lo; r0 < r_hi; r0 += 1024 * UN) {
            uint32_t w[UN];
            int act[UN];
            float olp[UN], G[UN];
#pragma unroll
            for (int k = 0; k < UN; k++) {
                const size_t c = gc + (size_t)min(r0 + 1024 * k + tid, r_hi - 1);
                w[k] = p.key_idx[c];
                act[k] = p.key_act[c];
                olp[k] = p.key_olp[c];
                G[k] = p.key_ret[c];
            }
            int rank[UN];
#pragma unroll
            for (int k = 0; k < UN; k++) rank[k] = p.key_rank[gd + w[k]];
#pragma unroll
            for (int k = 0; k < UN; k++) {
                const long long r = r0 + 1024 * k + tid;
                if (r >= r_hi || rank[k] < lo || rank[k] >= hi) continue;
                const float* fw = p.key_fwd + (gr + rank[k]) * KF;
                const bool av = (unsigned)act[k] < (unsigned)p.A;
                const float lp = av ? fw[act[k]] : 0.f;
                const float V = fw[16 * NT], ent = fw[16 * NT + 1];
                // the tile path's per-row derivatives with the rank's forward values
                const float ratio = fast_exp(lp - olp[k]);
                const float adv = G[k] - V;
                const float sur1 = ratio * adv;
                const float rc = fminf(fmaxf(ratio, 1.f - p.eps_clip), 1.f + p.eps_clip);
                const float sur2 = rc * adv;
                const float inr = (ratio >= 1.f - p.eps_clip && ratio <= 1.f + p.eps_clip) ? 1.f : 0.f;
                const float dmin = sur1 < sur2 ? adv : (sur2 < sur1 ? adv * inr : 0.5f * adv + 0.5f * adv * inr);
                const float qd = dmin * ratio, dv = V - G[k];
                if (!(fabsf(qd) <= p.key_bound && fabsf(dv) <= p.key_bound)) {  // NaN included
                    bad = true;
                    continue;
                }
                long long* a = sacc + (size_t)(rank[k] - lo) * KA;
                if (av) atomicAdd(reinterpret_cast<unsigned long long*>(a + act[k]), (unsigned long long)__float2ll_rn(qd * fx));
                atomicAdd(reinterpret_cast<unsigned long long*>(a + 16 * NT), (unsigned long long)__float2ll_rn(dv * fx));
                atomicAdd(scnt + (rank[k] - lo), 1u);
                l_min += -fminf(sur1, sur2);
                l_mse += dv * dv;
                l_ent += ent;
            }
        }
        __syncthreads();
        long long* dst = p.key_part + (pb * kKeyMaxRanks + lo) * KA;
        for (int i = tid; i < nr * KA; i += 1024) dst[i] = sacc[i];
        uint32_t* dc = p.key_pcnt + pb * kKeyMaxRanks + lo;
        for (int i = tid; i < nr; i += 1024) dc[i] = scnt[i];
        __syncthreads();
    }
    if (bad) __hip_atomic_store(p.key_flag + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the block's loss sums (fixed tree order)
    red[0][tid] = l_min;
    red[1][tid] = l_mse;
    red[2][tid] = l_ent;
    __syncthreads();
    for (int d = 512; d > 0; d >>= 1) {
        if (tid < d)
            for (int c = 0; c < 3; c++) red[c][tid] += red[c][tid + d];
        __syncthreads();
    }
    if (tid < 3) p.key_ploss[pb * 4 + tid] = red[tid][0];
}

// compact rows of many groups: the common row's forward per group, the row scan over all groups,
// the common sums per group, then the tiles of the marked rows (+ the virtual tile)
template <int NQ, int NT, int X = 0>
static hipError_t launch_own(const PpoArgs& a, unsigned nb, hipStream_t st) {
    hipError_t e;
    if ((e = launch_grad_cm<NQ, NT, kCommonFwd | X>(a, 1, st)) != hipSuccess) return e;
    const size_t lds = (size_t)a.A * 64 * (8 + 4) + 2 * 64 * 4;
    hipLaunchKernelGGL(k_own_scan, dim3((unsigned)a.own_nb, (unsigned)((a.G + 63) / 64)), dim3(256), lds, st, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_own_common, dim3((unsigned)a.G), dim3(256), 0, st, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return launch_grad_cm<NQ, NT, kMaskRow | X>(a, nb, st);
}

// MS_KEY_GATHER_ROWS=0: the per-lane gather for every layout (A/B measurements)
static bool gather_per_row() {
    static const bool v = [] {
        const char* e = getenv("MS_KEY_GATHER_ROWS");
        return e && e[0] == '0';
    }();
    return v;
}

// the common-row path for inputs up to 128 bytes (its scan holds a row per lane in registers)
// X = kX1: the tile path with a single-action last tile (A = 16 (NT - 1) + 1); the keyed passes never take it
template <int NQ, int NT, int X = 0>
static hipError_t launch_grad_t(const PpoArgs& a0, hipStream_t st) {
    PpoArgs a = a0;
    const unsigned nb = (unsigned)(a.n_chunks / 4);
    a.part_off = 0;
    if constexpr (NQ == 1 && NT <= 2) {
        if (a.key_mark && a.stride == 4 && !a.common) {
            // keyed rows: mark -> rank -> forward of the ranks -> row scan -> backward of the ranks,
            // then the tile path for the groups the keyed passes could not take
            hipError_t e;
            {
                const size_t n16 = (size_t)a.G * kKeyDense / 16;
                const unsigned cb = (unsigned)std::min<size_t>((n16 + 255) / 256, 4096);
                hipLaunchKernelGGL(k_key_clear, dim3(cb), dim3(256), 0, st, reinterpret_cast<uint4*>(a.key_mark), n16,
                                   a.key_flag, a.G);
                if ((e = hipGetLastError()) != hipSuccess) return e;
            }
            const unsigned ib = (unsigned)std::min<long long>((a.R + 255) / 256, 16384);
            if (a.rus == 1 && a.rrs <= 64 && (a.rrs & 3) == 0 && a.ret_ld <= 64 && a.ret_ld >= a.G &&
                !gather_per_row()) {
                const size_t lds = (size_t)kGatherWaves * 64 * (std::max<long long>(a.rrs, a.ret_ld) + 1) * 4;
                hipLaunchKernelGGL(k_key_gather_rows, dim3(ib), dim3(64 * kGatherWaves), lds, st, a);
            } else {
                hipLaunchKernelGGL(k_key_gather, dim3(ib), dim3(256), 0, st, a);
            }
            if ((e = hipGetLastError()) != hipSuccess) return e;
            hipLaunchKernelGGL(k_key_rank, dim3(a.G), dim3(1024), 0, st, a);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            a.part_rows = kKeyBlocks + (int)nb;
            if ((e = launch_grad_cm<NQ, NT, kKeyFwd>(a, kKeyBlocks, st)) != hipSuccess) return e;
            constexpr int KA = 16 * NT + 1;
            const size_t lds = (size_t)a.key_cap * (KA * 8 + 4);
            hipLaunchKernelGGL(k_key_scan<NT>, dim3((unsigned)(a.G * a.key_nbs)), dim3(1024), lds, st, a);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            if ((e = launch_grad_cm<NQ, NT, kKeyBack>(a, kKeyBlocks, st)) != hipSuccess) return e;
            a.part_off = kKeyBlocks;
            return launch_grad_cm<NQ, NT, kPlain>(a, nb, st);
        }
    }
    a.key_n = nullptr;
    a.part_rows = (int)nb;
    if constexpr (NQ <= 8) {
        if (a.common && a.stride >= 16) {
            using L = GradLds<NQ, NT, kCommonRow>;
            if (sizeof(float) * L::lds_floats <= 160 * 1024) {
                if (a.owner && a.own_mask && a.G >= kOwnMinGroups) return launch_own<NQ, NT, X>(a, nb, st);
                if (a.owner) return launch_grad_cm<NQ, NT, kOwnerRow | X>(a, nb, st);
                return launch_grad_cm<NQ, NT, kCommonRow | X>(a, nb, st);
            }
        }
    }
    if (a.owner) return hipErrorInvalidValue;  // compact rows need the common-row path
    return launch_grad_cm<NQ, NT, kPlain | X>(a, nb, st);
}

// MS_GRAD_X1=0: single-action last tiles on the MFMA like the others (A/B measurements)
static bool grad_x1_enabled() {
    static const bool v = [] {
        const char* e = getenv("MS_GRAD_X1");
        return !(e && e[0] == '0');
    }();
    return v;
}

// partial vectors per group that launch_ppo_grad writes (the keyed path adds its slot blocks)
int ppo_partial_rows(int n_chunks, bool keyed) { return n_chunks / 4 + (keyed ? kKeyBlocks : 0); }

hipError_t launch_ppo_grad(const PpoArgs& a, const GradOut& go, hipStream_t st) {
    const int nq = a.D / 16 + 1;  // 16*NQ > D leaves room for the ones column
    const int nt = (a.A + 15) / 16;
    if (a.n_chunks % 4 != 0) return hipErrorInvalidValue;
    hipError_t e;
    const bool keyed = a.key_mark && a.stride == 4 && !a.common && nq == 1 && nt <= 2;
#define MS_PPO_CASE(Q, T)                \
    if (nq <= Q && nt <= T) {            \
        e = launch_grad_t<Q, T>(a, st);  \
        goto reduce;                     \
    }
    // A = 16 (nt - 1) + 1 at the BASELINE shapes that have it (cfg4: offers C + 1 = 17 with 16 < D + 1 <= 64,
    // divided acceptors O + 1 = 49 with 64 < D + 1 <= 128)
    if (a.A % 16 == 1 && !keyed && grad_x1_enabled()) {
        if (nt == 2 && nq > 2 && nq <= 4) {
            e = launch_grad_t<4, 2, kX1>(a, st);
            goto reduce;
        }
        if (nt == 4 && nq > 4 && nq <= 8) {
            e = launch_grad_t<8, 4, kX1>(a, st);
            goto reduce;
        }
    }
    if (nt <= 1) {
        MS_PPO_CASE(1, 1) MS_PPO_CASE(2, 1) MS_PPO_CASE(4, 1) MS_PPO_CASE(8, 1) MS_PPO_CASE(16, 1)
    } else if (nt <= 2) {
        MS_PPO_CASE(1, 2) MS_PPO_CASE(2, 2) MS_PPO_CASE(4, 2) MS_PPO_CASE(8, 2) MS_PPO_CASE(16, 2)
    } else if (nt <= 4) {
        MS_PPO_CASE(2, 4) MS_PPO_CASE(4, 4) MS_PPO_CASE(8, 4) MS_PPO_CASE(16, 4)
    } else {
        MS_PPO_CASE(4, 8) MS_PPO_CASE(8, 8) MS_PPO_CASE(16, 8)
    }
#undef MS_PPO_CASE
    return hipErrorInvalidValue;
reduce:
    if (e != hipSuccess) return e;
    {
        const int P = poff(a.D, a.A).total;
        hipLaunchKernelGGL(k_ppo_reduce, dim3((P + 63) / 64, a.G), dim3(256), 0, st, a.partials, a.G,
                           ppo_partial_rows(a.n_chunks, keyed), P, a.D, a.A, go, keyed ? a.key_n : nullptr,
                           keyed ? a.key_flag : nullptr, kKeyBlocks);
    }
    return hipGetLastError();
}

int ppo_param_count(int D, int A) { return poff(D, A).total; }
}  // namespace ms
#ifdef MS_GRAD_PROBE
extern "C" int ms_grad_probe_read(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ms::g_grad_probe), bytes, 0, hipMemcpyDeviceToHost);
}
#endif
namespace ms {

// ---------------------------------------------------------------------------
// Adam (torch.optim.Adam's foreach step, torch/optim/adam.py _multi_tensor_adam) over up to 16
// tensors of one PPO group in one launch: blockIdx.y = tensor. Per element, each foreach op's
// f32 rounding in turn:
//   m = lerp(m, g, 1 - beta1);  v = v * beta2 + (1 - beta2) * g * g;
//   p += (-lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
struct AdamArgs {
    AdamTensor t[kAdamMaxTensors];
    float w1, beta2, one_m_beta2, eps;
    float neg_step[kAdamMaxGroups], bc2_sqrt;
    // device step counter (HIP-graph replays): the bias corrections from *step_dev, computed as
    // launch_adam computes them on the host
    const int64_t* step_dev;
    double lr[kAdamMaxGroups], beta1d, beta2d;
};

__global__ void __launch_bounds__(256) k_adam(AdamArgs a) {
    const AdamTensor& t = a.t[blockIdx.y];
    float ns = a.neg_step[t.lr_group], bc2_sqrt = a.bc2_sqrt;
    if (a.step_dev) {
        const double step = (double)*a.step_dev;
        const double bc1 = 1.0 - pow(a.beta1d, step), bc2 = 1.0 - pow(a.beta2d, step);
        ns = (float)((a.lr[t.lr_group] / bc1) * -1.0);
        bc2_sqrt = (float)sqrt(bc2);
    }
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < t.numel; i += (int64_t)gridDim.x * 256) {
        const float g = t.grad[i];
        float m = t.exp_avg[i], v = t.exp_avg_sq[i];
        m = m + a.w1 * (g - m);                  // lerp, weight < 0.5
        v = v * a.beta2;                         // mul_
        v = v + a.one_m_beta2 * (g * g);         // addcmul_
        const float den = sqrtf(v) / bc2_sqrt + a.eps;
        t.param[i] = t.param[i] + ns * (m / den);  // addcdiv_
        t.exp_avg[i] = m;
        t.exp_avg_sq[i] = v;
    }
}

hipError_t launch_adam(const AdamTensor* ts, int n, const double* lr, int n_lr, int64_t step, double beta1,
                       double beta2, double eps, const int64_t* step_dev, hipStream_t st) {
    if (n < 1 || n > kAdamMaxTensors || n_lr < 1 || n_lr > kAdamMaxGroups || (step < 1 && !step_dev))
        return hipErrorInvalidValue;
    if (step_dev) step = 1;  // the host-side corrections are unused
    AdamArgs a{};
    a.step_dev = step_dev;
    a.beta1d = beta1;
    a.beta2d = beta2;
    for (int k = 0; k < n_lr; k++) a.lr[k] = lr[k];
    int64_t mx = 1;
    for (int i = 0; i < n; i++) {
        if (ts[i].lr_group < 0 || ts[i].lr_group >= n_lr) return hipErrorInvalidValue;
        a.t[i] = ts[i];
        mx = ts[i].numel > mx ? ts[i].numel : mx;
    }
    // the scalars as torch computes them (Python floats) and passes them to the f32 foreach ops
    const double bc1 = 1.0 - pow(beta1, (double)step), bc2 = 1.0 - pow(beta2, (double)step);
    a.w1 = (float)(1.0 - beta1);
    a.beta2 = (float)beta2;
    a.one_m_beta2 = (float)(1.0 - beta2);
    a.eps = (float)eps;
    for (int k = 0; k < n_lr; k++) a.neg_step[k] = (float)((lr[k] / bc1) * -1.0);
    a.bc2_sqrt = (float)sqrt(bc2);
    int64_t bx = (mx + 255) / 256;
    bx = bx > 1024 ? 1024 : bx;
    hipLaunchKernelGGL(k_adam, dim3((unsigned)bx, (unsigned)n), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace ms
