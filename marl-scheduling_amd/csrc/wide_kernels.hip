// wide_kernels.hip — the aggregated agents' ActorCritics (PPOmodules.py:177-232) on gfx950: act and
// the PPO gradient for 32 / 64 hidden units and action counts from a handful to tens of thousands
// ((O+1)^C acceptor numbers, (C+1)^L offer numbers, their product for the fully aggregated net).
//
// The 16-wide policy kernels keep a row's logits in registers; here a row has up to A logits, so a
// block of 256 threads takes a tile of 16 rows of one group (agent net) and every thread owns a
// contiguous chunk of ceil(A / 256) actions for all 16 rows. Per-row statistics over the actions
// are block reductions in a fixed order (deterministic); the sample is an inverse CDF over the
// chunks (block scan of the chunk sums).
//
//   k_wide_act     ActorCritic.act (PPOmodules.py:53-63): tanh MLP, softmax, Categorical sample at
//                  a given uniform (the action is the number of running sums <= u * S) and its
//                  log-prob log(clamp(p_a)), for rows (e, g) of [E][G][stride] int8 observations;
//   k_wide_rows    PPO.update's per-row work (PPOmodules.py:144-168): forward of actor and critic,
//                  the softmax + Categorical renormalisation + clamped-log statistics, the loss
//                  derivatives of -min(surr) + 0.5 MSE - 0.01 entropy, d logits (gz) and the
//                  backward through both MLPs to every layer's pre-activation gradient. The
//                  logits of the tile live in a per-block scratch [16][A]; the row's activations,
//                  pre-activation gradients and statistics go to a row record;
//   k_wide_outer   the hidden layers' weight gradients as batch reductions over the records,
//                  dW = sum_r d_r (x) v_r (+ the bias column), one block per (layer, row split,
//                  group), threads split over output columns and row phases;
//   k_wide_w3      the output layer's gradient dW3 = sum_r gz_r (x) h2_r: a lane per action
//                  recomputes gz from the row's logit and statistics (the same arithmetic as
//                  k_wide_rows) instead of materialising [R][A];
//   k_wide_reduce  the row splits' partial gradients summed in split order into the gradient
//                  tensors, and the block loss partials into the per-group means.
//
// Arithmetic follows torch's f32 formulas (softmax exp(z - max) / sum, Categorical's p / sum(p),
// log(clamp(p, eps, 1 - eps))); sums run in a different order than torch's, so the gradient
// agrees with autograd to f32 rounding (tests/test_wide_gpu.py).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "ms_wide.h"

namespace ms {
namespace {

constexpr int TPB = kWideThreads;
constexpr int TR = kWideRowsPerTile;
constexpr float kEps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps (probs_to_logits clamp)

__device__ __forceinline__ float clampp(float p) { return fminf(fmaxf(p, kEps), 1.f - kEps); }

template <typename T, bool MAX>
__device__ __forceinline__ T wave_red(T v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const T o = __shfl_xor(v, m, 64);
        v = MAX ? (o > v ? o : v) : v + o;  // commutative: every lane ends with the same value
    }
    return v;
}

// Sum (or max) over the block's 256 threads of NV values per thread -> out[i], i < NV (LDS).
// red: [4][NV] scratch. Ends with a barrier.
template <typename T, int NV, bool MAX>
__device__ __forceinline__ void block_red(T (&v)[NV], T* red, T* out, int t) {
#pragma unroll
    for (int i = 0; i < NV; i++) v[i] = wave_red<T, MAX>(v[i]);
    if ((t & 63) == 0)
#pragma unroll
        for (int i = 0; i < NV; i++) red[(t >> 6) * NV + i] = v[i];
    __syncthreads();
    if (t < NV) {
        const T a = red[t], b = red[NV + t], c = red[2 * NV + t], d = red[3 * NV + t];
        if constexpr (MAX) {
            const T ab = a > b ? a : b, cd = c > d ? c : d;
            out[t] = ab > cd ? ab : cd;
        } else {
            out[t] = (a + b) + (c + d);
        }
    }
    __syncthreads();
}

// out[r][j] = tanh(b[j] + W[j] . in[r]) for the tile's 16 rows and H outputs (two nets at once:
// net 1 writes out1, net 2 out2; W1 / W2 [H][K] row-major like torch's Linear weight)
template <int H>
__device__ __forceinline__ void dense2(const float* Wa, const float* ba, const float* Wb, const float* bb, int K,
                                       const float* in_a, const float* in_b, int ip, float* out_a, float* out_b,
                                       int op, int t) {
    for (int i = t; i < 2 * TR * H; i += TPB) {
        const int net = i / (TR * H), rem = i % (TR * H), r = rem % TR, j = rem / TR;
        const float* w = (net ? Wb : Wa) + (size_t)j * K;
        const float* x = (net ? in_b : in_a) + r * ip;
        float acc = 0.f;
        for (int k = 0; k < K; k++) acc = fmaf(w[k], x[k], acc);
        (net ? out_b : out_a)[r * op + j] = tanhf(acc + (net ? bb : ba)[j]);
    }
}

template <int H>
__device__ __forceinline__ void dense1(const float* W, const float* b, int K, const float* in, int ip, float* out, int op,
                                       int t) {
    for (int i = t; i < TR * H; i += TPB) {
        const int r = i % TR, j = i / TR;
        const float* w = W + (size_t)j * K;
        const float* x = in + r * ip;
        float acc = 0.f;
        for (int k = 0; k < K; k++) acc = fmaf(w[k], x[k], acc);
        out[r * op + j] = tanhf(acc + b[j]);
    }
}

// int8 rows of the tile as f32, zeros past D and for rows beyond the batch
__device__ __forceinline__ void load_rows(float* sx, int xp, const int8_t* base, long long row0, long long nrows, int G,
                                          int g, int stride, int D, int t) {
    for (int i = t; i < TR * D; i += TPB) {
        const int r = i / D, k = i % D;
        float v = 0.f;
        if (row0 + r < nrows) v = (float)base[((row0 + r) * G + g) * (long long)stride + k];
        sx[r * xp + k] = v;
    }
}

// logit of action a for one row: W3 row a (registers) . h2 (LDS, 16-byte aligned) + b3[a]
template <int H>
__device__ __forceinline__ float logit(const float (&w)[H], const float* h, float b) {
    float acc = 0.f;
#pragma unroll
    for (int k4 = 0; k4 < H / 4; k4++) {
        const float4 hv = *reinterpret_cast<const float4*>(h + 4 * k4);
        acc = fmaf(w[4 * k4 + 0], hv.x, acc);
        acc = fmaf(w[4 * k4 + 1], hv.y, acc);
        acc = fmaf(w[4 * k4 + 2], hv.z, acc);
        acc = fmaf(w[4 * k4 + 3], hv.w, acc);
    }
    return acc + b;
}

// W3 row a into registers. The compiler barrier keeps the per-row h2 reads that follow inside
// the action loop (16 rows x H floats of LDS, loop-invariant) from being hoisted into registers.
template <int H>
__device__ __forceinline__ void load_w(float (&w)[H], const float* row) {
    __asm__ volatile("" ::: "memory");
#pragma unroll
    for (int k4 = 0; k4 < H / 4; k4++) {
        const float4 v = *reinterpret_cast<const float4*>(row + 4 * k4);
        w[4 * k4 + 0] = v.x;
        w[4 * k4 + 1] = v.y;
        w[4 * k4 + 2] = v.z;
        w[4 * k4 + 3] = v.w;
    }
}

// d loss / d pn_a of one (row, action) given the softmax output pe_a: the log-prob term (action
// taken) and the entropy term -sum cl * pn, through log(clamp(pn)); also returns pn and cl
__device__ __forceinline__ float dpn_of(float pe, bool taken, float inv1, float g_lp, float g_h, float& pn, float& cl) {
    pn = pe * inv1;
    const float cp = clampp(pn);
    cl = logf(cp);
    const float in = (pn >= kEps && pn <= 1.f - kEps) ? 1.f : 0.f;
    const float dl = taken ? g_lp : 0.f;
    return (dl - g_h * pn) * in / cp - g_h * cl;
}

// d loss / d pe through the renormalisation pn = pe / sum(pe), before the softmax backward
__device__ __forceinline__ float dpe_of(float v, float x1, float inv1) { return (v - x1 * inv1) * inv1; }

// d loss / d z through the softmax
__device__ __forceinline__ float dz_of(float pe, float gzp, float x2) { return pe * (gzp - x2); }

__device__ __forceinline__ void chunk_of(int A, int t, int& a0, int& a1) {
    const int c = (A + TPB - 1) / TPB;
    a0 = t * c < A ? t * c : A;
    a1 = a0 + c < A ? a0 + c : A;
}

__host__ __device__ constexpr int pitch_h(int H) { return H + 4; }   // 16-byte rows, 16 lanes x 4 j conflict-free
__host__ __device__ constexpr int pitch_x(int D) { return D | 1; }   // odd: 16 rows on distinct banks
__host__ __device__ constexpr int up4(int n) { return (n + 3) & ~3; }

// ---------------------------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(TPB) void k_wide_act(WideAct p) {
    extern __shared__ float lds[];
    constexpr int HP = pitch_h(H);
    const int t = threadIdx.x, g = blockIdx.y, D = p.D, A = p.A;
    const long long e0 = (long long)blockIdx.x * TR;
    const int xp = pitch_x(D);
    float* sx = lds;
    float* sh1 = sx + up4(TR * xp);
    float* sh2 = sh1 + TR * HP;
    float* sM = sh2 + TR * HP;
    float* sS = sM + TR;
    float* red = sS + TR;  // [4][16]
    float* wtot = red + 4 * TR;  // [4][16]
    int* ired = reinterpret_cast<int*>(wtot + 4 * TR);  // [4][16]
    int* sLast = ired + 4 * TR;
    int* sCnt = sLast + TR;

    const WideNet& n = p.actor;
    const float* w1 = n.w1 + (size_t)g * H * D;
    const float* b1 = n.b1 + (size_t)g * H;
    const float* w2 = n.w2 + (size_t)g * H * H;
    const float* b2 = n.b2 + (size_t)g * H;
    const float* w3 = n.w3 + (size_t)g * A * H;
    const float* b3 = n.b3 + (size_t)g * A;

    load_rows(sx, xp, p.obs, e0, p.E, p.G, g, p.stride, D, t);
    __syncthreads();
    dense1<H>(w1, b1, D, sx, xp, sh1, HP, t);
    __syncthreads();
    dense1<H>(w2, b2, H, sh1, HP, sh2, HP, t);
    __syncthreads();

    int a0, a1;
    chunk_of(A, t, a0, a1);
    float w[H];
    // pass 1: row maxima
    float m[TR];
#pragma unroll
    for (int r = 0; r < TR; r++) m[r] = -INFINITY;
    for (int a = a0; a < a1; a++) {
        load_w<H>(w, w3 + (size_t)a * H);
        const float b = b3[a];
#pragma unroll
        for (int r = 0; r < TR; r++) m[r] = fmaxf(m[r], logit<H>(w, sh2 + r * HP, b));
    }
    block_red<float, TR, true>(m, red, sM, t);
    // pass 2: chunk sums of exp(z - max) and the last action with a nonzero term
    float s[TR], sc[TR];
    int last[TR];
#pragma unroll
    for (int r = 0; r < TR; r++) {
        s[r] = 0.f;
        last[r] = -1;
    }
    for (int a = a0; a < a1; a++) {
        load_w<H>(w, w3 + (size_t)a * H);
        const float b = b3[a];
#pragma unroll
        for (int r = 0; r < TR; r++) {
            const float e = expf(logit<H>(w, sh2 + r * HP, b) - sM[r]);
            s[r] += e;
            if (e > 0.f) last[r] = a;
        }
    }
#pragma unroll
    for (int r = 0; r < TR; r++) sc[r] = s[r];
    block_red<float, TR, false>(s, red, sS, t);
    block_red<int, TR, true>(last, ired, sLast, t);
    // exclusive prefix of the chunk sums in action order (thread order)
    const int lane = t & 63, wv = t >> 6;
    float pre[TR];
#pragma unroll
    for (int r = 0; r < TR; r++) {
        float v = sc[r];
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const float o = __shfl_up(v, off, 64);
            if (lane >= off) v += o;
        }
        const float ex = __shfl_up(v, 1, 64);
        pre[r] = lane ? ex : 0.f;
        if (lane == 63) wtot[wv * TR + r] = v;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < TR; r++) {
        float base = 0.f;
        for (int q = 0; q < wv; q++) base += wtot[q * TR + r];
        pre[r] += base;
    }
    // pass 3: count the running sums <= u * S
    int cnt[TR];
    float target[TR];
#pragma unroll
    for (int r = 0; r < TR; r++) {
        cnt[r] = 0;
        const long long e = e0 + r;
        target[r] = (e < p.E ? p.uniforms[e * p.G + g] : 0.f) * sS[r];
    }
    for (int a = a0; a < a1; a++) {
        load_w<H>(w, w3 + (size_t)a * H);
        const float b = b3[a];
#pragma unroll
        for (int r = 0; r < TR; r++) {
            pre[r] += expf(logit<H>(w, sh2 + r * HP, b) - sM[r]);
            cnt[r] += pre[r] <= target[r] ? 1 : 0;
        }
    }
    block_red<int, TR, false>(cnt, ired, sCnt, t);
    if (t < TR && e0 + t < p.E) {
        int act = sCnt[t];
        if (act >= A) act = sLast[t] >= 0 ? sLast[t] : A - 1;  // u * S at or beyond the rounded total
        load_w<H>(w, w3 + (size_t)act * H);
        const float e = expf(logit<H>(w, sh2 + t * HP, b3[act]) - sM[t]);
        const float pe = e * (1.f / sS[t]);
        const long long o = (e0 + t) * p.G + g;
        p.action[o] = act;
        p.logprob[o] = logf(clampp(pe));
    }
}

// ---------------------------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(TPB) void k_wide_rows(WideRows p) {
    extern __shared__ float lds[];
    constexpr int HP = pitch_h(H);
    constexpr int RW = 8 * H + kWideStats;
    constexpr int RG = TPB / H;   // row groups of the hidden-unit-parallel steps
    constexpr int RPT = TR / RG;  // rows per thread there
    const int t = threadIdx.x, g = blockIdx.y, b = blockIdx.x, D = p.D, A = p.A;
    const int xp = pitch_x(D);
    float* sx = lds;
    float* sh1 = sx + up4(TR * xp);
    float* sh2 = sh1 + TR * HP;
    float* shc1 = sh2 + TR * HP;
    float* shc2 = shc1 + TR * HP;
    float* sd1 = shc2 + TR * HP;
    float* sd2 = sd1 + TR * HP;
    float* sc1 = sd2 + TR * HP;
    float* sc2 = sc1 + TR * HP;
    float* sM = sc2 + TR * HP;
    float* sS = sM + TR;
    float* sP1 = sS + TR;
    float* sX1 = sP1 + TR;  // [32]: x1 then entropy
    float* sX2 = sX1 + 2 * TR;
    float* sV = sX2 + TR;
    float* sRet = sV + TR;
    float* sOlp = sRet + TR;
    float* sGlp = sOlp + TR;
    float* sGh = sGlp + TR;
    float* sGv = sGh + TR;
    float* sL = sGv + TR;  // [3][16] loss partials
    float* red = sL + 3 * TR;  // [4][32]
    int* sAct = reinterpret_cast<int*>(red + 4 * 2 * TR);

    const WideNet& an = p.actor;
    const WideNet& cn = p.critic;
    const float* aw1 = an.w1 + (size_t)g * H * D;
    const float* ab1 = an.b1 + (size_t)g * H;
    const float* aw2 = an.w2 + (size_t)g * H * H;
    const float* ab2 = an.b2 + (size_t)g * H;
    const float* aw3 = an.w3 + (size_t)g * A * H;
    const float* ab3 = an.b3 + (size_t)g * A;
    const float* cw1 = cn.w1 + (size_t)g * H * D;
    const float* cb1 = cn.b1 + (size_t)g * H;
    const float* cw2 = cn.w2 + (size_t)g * H * H;
    const float* cb2 = cn.b2 + (size_t)g * H;
    const float* cw3 = cn.w3 + (size_t)g * H;
    const float cb3 = cn.b3[g];
    float* zb = p.zbuf + ((size_t)g * p.NB + b) * TR * (size_t)A;

    float l_min = 0.f, l_mse = 0.f, l_ent = 0.f;  // thread r < 16: its rows' loss terms
    int a0, a1;
    chunk_of(A, t, a0, a1);
    float w[H];
    const long long ntiles = (p.R + TR - 1) / TR;
    for (long long tile = b; tile < ntiles; tile += p.NB) {
        const long long row0 = tile * TR;
        const int nv = (int)(p.R - row0 < TR ? p.R - row0 : TR);
        load_rows(sx, xp, p.states, row0, p.R, p.G, g, p.stride, D, t);
        if (t < TR) {
            int act = 0;
            float olp = 0.f, ret = 0.f;
            if (t < nv) {
                const long long o = (row0 + t) * p.G + g;
                act = p.actions[o];
                act = act < 0 ? 0 : (act >= A ? A - 1 : act);
                olp = p.old_logprob[o];
                ret = p.returns[(long long)g * p.R + row0 + t];
            }
            sAct[t] = act;
            sOlp[t] = olp;
            sRet[t] = ret;
        }
        __syncthreads();
        dense2<H>(aw1, ab1, cw1, cb1, D, sx, sx, xp, sh1, shc1, HP, t);
        __syncthreads();
        dense2<H>(aw2, ab2, cw2, cb2, H, sh1, shc1, HP, sh2, shc2, HP, t);
        __syncthreads();
        if (t < TR) {
            float v = 0.f;
            for (int k = 0; k < H; k++) v = fmaf(cw3[k], shc2[t * HP + k], v);
            sV[t] = v + cb3;
        }
        // pass 1: logits -> scratch, row maxima
        float v16[TR];
#pragma unroll
        for (int r = 0; r < TR; r++) v16[r] = -INFINITY;
        for (int a = a0; a < a1; a++) {
            load_w<H>(w, aw3 + (size_t)a * H);
            const float bb = ab3[a];
#pragma unroll
            for (int r = 0; r < TR; r++) {
                const float z = logit<H>(w, sh2 + r * HP, bb);
                zb[r * A + a] = z;
                v16[r] = fmaxf(v16[r], z);
            }
        }
        block_red<float, TR, true>(v16, red, sM, t);
        // pass 2: e = exp(z - max), S
#pragma unroll
        for (int r = 0; r < TR; r++) v16[r] = 0.f;
        for (int a = a0; a < a1; a++)
#pragma unroll
            for (int r = 0; r < TR; r++) {
                const float e = expf(zb[r * A + a] - sM[r]);
                zb[r * A + a] = e;
                v16[r] += e;
            }
        block_red<float, TR, false>(v16, red, sS, t);
        // pass 3: softmax output pe = e / S, sum(pe)
#pragma unroll
        for (int r = 0; r < TR; r++) v16[r] = 0.f;
        for (int a = a0; a < a1; a++)
#pragma unroll
            for (int r = 0; r < TR; r++) {
                const float pe = zb[r * A + a] * (1.f / sS[r]);
                zb[r * A + a] = pe;
                v16[r] += pe;
            }
        block_red<float, TR, false>(v16, red, sP1, t);
        // per-row loss derivatives (loss.mean() over R rows)
        if (t < TR) {
            const float inv1 = 1.f / sP1[t];
            const float lp = logf(clampp(zb[t * A + sAct[t]] * inv1));
            const float V = sV[t], G = sRet[t];
            const float ratio = expf(lp - sOlp[t]);
            const float adv = G - V;
            const float sur1 = ratio * adv;
            const float rc = fminf(fmaxf(ratio, 1.f - p.eps_clip), 1.f + p.eps_clip);
            const float sur2 = rc * adv;
            const float inr = (ratio >= 1.f - p.eps_clip && ratio <= 1.f + p.eps_clip) ? 1.f : 0.f;
            // d min(s1, s2) / d ratio (torch.minimum splits ties)
            const float dmin = sur1 < sur2 ? adv : (sur2 < sur1 ? adv * inr : 0.5f * adv + 0.5f * adv * inr);
            const bool valid = t < nv;
            const float wgt = valid ? p.inv_R : 0.f;
            sGlp[t] = -dmin * wgt * ratio;
            sGv[t] = (V - G) * wgt;
            sGh[t] = -0.01f * wgt;
            if (valid) {
                l_min += -fminf(sur1, sur2);
                l_mse += (V - G) * (V - G);
            }
        }
        __syncthreads();
        // pass 4: x1 = sum v * pe and the entropy -sum cl * pn
        float x1e[2 * TR];
#pragma unroll
        for (int r = 0; r < 2 * TR; r++) x1e[r] = 0.f;
        for (int a = a0; a < a1; a++)
#pragma unroll
            for (int r = 0; r < TR; r++) {
                const float pe = zb[r * A + a];
                float pn, cl;
                const float v = dpn_of(pe, a == sAct[r], 1.f / sP1[r], sGlp[r], sGh[r], pn, cl);
                x1e[r] += v * pe;
                x1e[TR + r] -= cl * pn;
            }
        block_red<float, 2 * TR, false>(x1e, red, sX1, t);
        if (t < TR && t < nv) l_ent += sX1[TR + t];
        // pass 5: x2 = sum gzp * pe
#pragma unroll
        for (int r = 0; r < TR; r++) v16[r] = 0.f;
        for (int a = a0; a < a1; a++)
#pragma unroll
            for (int r = 0; r < TR; r++) {
                const float pe = zb[r * A + a];
                const float inv1 = 1.f / sP1[r];
                float pn, cl;
                const float v = dpn_of(pe, a == sAct[r], inv1, sGlp[r], sGh[r], pn, cl);
                v16[r] += dpe_of(v, sX1[r], inv1) * pe;
            }
        block_red<float, TR, false>(v16, red, sX2, t);
        // pass 6: gz -> scratch
        for (int a = a0; a < a1; a++)
#pragma unroll
            for (int r = 0; r < TR; r++) {
                const float pe = zb[r * A + a];
                const float inv1 = 1.f / sP1[r];
                float pn, cl;
                const float v = dpn_of(pe, a == sAct[r], inv1, sGlp[r], sGh[r], pn, cl);
                zb[r * A + a] = dz_of(pe, dpe_of(v, sX1[r], inv1), sX2[r]);
            }
        __syncthreads();
        // d h2 = W3^T gz (thread: hidden unit k, rows rg + RG i), d pre2; critic d pre2
        {
            const int k = t % H, rg = t / H;
            float acc[RPT];
#pragma unroll
            for (int i = 0; i < RPT; i++) acc[i] = 0.f;
            for (int a = 0; a < A; a++) {
                const float wk = aw3[(size_t)a * H + k];
#pragma unroll
                for (int i = 0; i < RPT; i++) acc[i] = fmaf(zb[(rg + RG * i) * A + a], wk, acc[i]);
            }
#pragma unroll
            for (int i = 0; i < RPT; i++) {
                const int r = rg + RG * i;
                const float h2 = sh2[r * HP + k], hc2 = shc2[r * HP + k];
                sd2[r * HP + k] = acc[i] * (1.f - h2 * h2);
                sc2[r * HP + k] = sGv[r] * cw3[k] * (1.f - hc2 * hc2);
            }
        }
        __syncthreads();
        // d h1 = W2^T d2 (thread: hidden unit j), d pre1; critic the same
        {
            const int j = t % H, rg = t / H;
            float acc[RPT], cacc[RPT];
#pragma unroll
            for (int i = 0; i < RPT; i++) acc[i] = cacc[i] = 0.f;
            for (int k = 0; k < H; k++) {
                const float wa = aw2[(size_t)k * H + j], wc = cw2[(size_t)k * H + j];
#pragma unroll
                for (int i = 0; i < RPT; i++) {
                    const int r = rg + RG * i;
                    acc[i] = fmaf(wa, sd2[r * HP + k], acc[i]);
                    cacc[i] = fmaf(wc, sc2[r * HP + k], cacc[i]);
                }
            }
#pragma unroll
            for (int i = 0; i < RPT; i++) {
                const int r = rg + RG * i;
                const float h1 = sh1[r * HP + j], hc1 = shc1[r * HP + j];
                sd1[r * HP + j] = acc[i] * (1.f - h1 * h1);
                sc1[r * HP + j] = cacc[i] * (1.f - hc1 * hc1);
            }
        }
        __syncthreads();
        // row records
        for (int i = t; i < nv * RW; i += TPB) {
            const int r = i / RW, c = i % RW, part = c / H, k = c % H;
            float v;
            if (part < 8) {
                const float* src = part == 0 ? sh1 : part == 1 ? sh2 : part == 2 ? shc1 : part == 3 ? shc2
                                 : part == 4 ? sd1 : part == 5 ? sd2 : part == 6 ? sc1 : sc2;
                v = src[r * HP + k];
            } else {
                const int s = c - 8 * H;
                v = s == kStM ? sM[r] : s == kStRS ? 1.f / sS[r] : s == kStInv1 ? 1.f / sP1[r] : s == kStX1 ? sX1[r]
                  : s == kStX2 ? sX2[r] : s == kStGlp ? sGlp[r] : s == kStGh ? sGh[r] : s == kStGv ? sGv[r]
                  : s == kStAct ? __int_as_float(sAct[r]) : 0.f;
            }
            p.rec[((size_t)g * p.R + row0 + r) * RW + c] = v;
        }
        __syncthreads();
    }
    // the block's loss partials, rows summed in thread order
    if (t < TR) {
        sL[t] = l_min;
        sL[TR + t] = l_mse;
        sL[2 * TR + t] = l_ent;
    }
    __syncthreads();
    if (t < 3) {
        float s = 0.f;
        for (int r = 0; r < TR; r++) s += sL[t * TR + r];
        p.loss_part[((size_t)g * p.NB + b) * 3 + t] = s;
    }
}

// ---------------------------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(TPB) void k_wide_outer(WideGrads p) {
    extern __shared__ float lds[];
    constexpr int RW = 8 * H + kWideStats;
    const int job = blockIdx.x, s = blockIdx.y, g = blockIdx.z, t = threadIdx.x;
    int M = H, N, uoff, voff = 0, ow, ob;
    bool vx = false;
    switch (job) {
        case 0: N = p.D; uoff = 4 * H; vx = true; ow = kOW1; ob = kOB1; break;      // d1 (x) x
        case 1: N = H; uoff = 5 * H; voff = 0; ow = kOW2; ob = kOB2; break;         // d2 (x) h1
        case 2: N = p.D; uoff = 6 * H; vx = true; ow = kOCW1; ob = kOCB1; break;    // c1 (x) x
        case 3: N = H; uoff = 7 * H; voff = 2 * H; ow = kOCW2; ob = kOCB2; break;   // c2 (x) hc1
        default: M = 1; N = H; uoff = 8 * H + kStGv; voff = 3 * H; ow = kOCW3; ob = kOCB3; break;  // g_v (x) hc2
    }
    const int NC = N + 1, P = TPB / NC, ph = t / NC, n = t % NC;
    const bool active = ph < P;
    float* sU = lds;             // [16][M]
    float* red = sU + TR * H;    // [P][M][NC]
    float acc[H];
#pragma unroll
    for (int m = 0; m < H; m++) acc[m] = 0.f;
    const long long r0 = (long long)s * p.rows_per_split;
    const long long r1 = r0 + p.rows_per_split < p.R ? r0 + p.rows_per_split : p.R;
    const float* rec = p.rec + (size_t)g * p.R * RW;
    for (long long row0 = r0; row0 < r1; row0 += TR) {
        const int nv = (int)(r1 - row0 < TR ? r1 - row0 : TR);
        for (int i = t; i < TR * M; i += TPB) {
            const int r = i / M, m = i % M;
            sU[r * M + m] = r < nv ? rec[(size_t)(row0 + r) * RW + uoff + m] : 0.f;
        }
        __syncthreads();
        if (active)
            for (int r = ph; r < nv; r += P) {
                float v = 1.f;
                if (n < N)
                    v = vx ? (float)p.states[((row0 + r) * p.G + g) * (long long)p.stride + n]
                           : rec[(size_t)(row0 + r) * RW + voff + n];
#pragma unroll
                for (int m = 0; m < H; m++)
                    if (m < M) acc[m] = fmaf(sU[r * M + m], v, acc[m]);
            }
        __syncthreads();
    }
    if (active)
#pragma unroll
        for (int m = 0; m < H; m++)
            if (m < M) red[(ph * M + m) * NC + n] = acc[m];
    __syncthreads();
    float* out = p.part + ((size_t)s * p.G + g) * p.off.o[kWideSegs];
    for (int i = t; i < M * NC; i += TPB) {
        const int m = i / NC, nn = i % NC;
        float sum = 0.f;
        for (int q = 0; q < P; q++) sum += red[(q * M + m) * NC + nn];
        out[nn < N ? p.off.o[ow] + (long long)m * N + nn : p.off.o[ob] + m] = sum;
    }
}

// ---------------------------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(TPB) void k_wide_w3(WideGrads p) {
    extern __shared__ float lds[];
    constexpr int HP = pitch_h(H);
    constexpr int RW = 8 * H + kWideStats;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, s = blockIdx.y, g = blockIdx.z, A = p.A;
    const int a = blockIdx.x * 64 + lane;
    const bool on = a < A;
    float* sh2 = lds;                  // [16][HP]
    float* sst = sh2 + TR * HP;        // [16][kWideStats]
    float* red = sst + TR * kWideStats;  // [4 * 64][H + 1]
    float w[H], acc[H], accb = 0.f;
    const float* w3 = p.actor.w3 + (size_t)g * A * H;
    float b3 = 0.f;
    if (on) {
        load_w<H>(w, w3 + (size_t)a * H);
        b3 = p.actor.b3[(size_t)g * A + a];
    } else {
#pragma unroll
        for (int k = 0; k < H; k++) w[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < H; k++) acc[k] = 0.f;
    const long long r0 = (long long)s * p.rows_per_split;
    const long long r1 = r0 + p.rows_per_split < p.R ? r0 + p.rows_per_split : p.R;
    const float* rec = p.rec + (size_t)g * p.R * RW;
    for (long long row0 = r0; row0 < r1; row0 += TR) {
        const int nv = (int)(r1 - row0 < TR ? r1 - row0 : TR);
        for (int i = t; i < TR * H; i += TPB) {
            const int r = i / H, k = i % H;
            sh2[r * HP + k] = r < nv ? rec[(size_t)(row0 + r) * RW + H + k] : 0.f;
        }
        for (int i = t; i < TR * kWideStats; i += TPB) {
            const int r = i / kWideStats;
            sst[i] = r < nv ? rec[(size_t)(row0 + r) * RW + 8 * H + i % kWideStats] : 0.f;
        }
        __syncthreads();
        if (on)
            for (int r = wv; r < nv; r += 4) {
                const float* st = sst + r * kWideStats;
                const float z = logit<H>(w, sh2 + r * HP, b3);
                const float pe = expf(z - st[kStM]) * st[kStRS];
                const float inv1 = st[kStInv1];
                float pn, cl;
                const float v = dpn_of(pe, a == __float_as_int(st[kStAct]), inv1, st[kStGlp], st[kStGh], pn, cl);
                const float gz = dz_of(pe, dpe_of(v, st[kStX1], inv1), st[kStX2]);
                accb += gz;
#pragma unroll
                for (int k = 0; k < H; k++) acc[k] = fmaf(gz, sh2[r * HP + k], acc[k]);
            }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < H; k++) red[(wv * 64 + lane) * (H + 1) + k] = acc[k];
    red[(wv * 64 + lane) * (H + 1) + H] = accb;
    __syncthreads();
    float* out = p.part + ((size_t)s * p.G + g) * p.off.o[kWideSegs];
    for (int i = t; i < 64 * (H + 1); i += TPB) {
        const int l = i / (H + 1), k = i % (H + 1), aa = blockIdx.x * 64 + l;
        if (aa >= A) continue;
        float sum = 0.f;
        for (int q = 0; q < 4; q++) sum += red[(q * 64 + l) * (H + 1) + k];
        out[k < H ? p.off.o[kOW3] + (long long)aa * H + k : p.off.o[kOB3] + aa] = sum;
    }
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(TPB) void k_wide_reduce(WideReduce p) {
    const long long total = p.off.o[kWideSegs];
    const long long i = (long long)blockIdx.x * TPB + threadIdx.x;
    if (i < (long long)p.G * total) {
        const long long g = i / total, e = i % total;
        float sum = 0.f;
        for (int s = 0; s < p.RS; s++) sum += p.part[((size_t)s * p.G + g) * total + e];
        int seg = 0;
        while (seg + 1 < kWideSegs && p.off.o[seg + 1] <= e) seg++;
        const long long cnt = p.off.o[seg + 1] - p.off.o[seg];
        p.dst[seg][g * cnt + (e - p.off.o[seg])] = sum;
    }
    if (blockIdx.x == 0)
        for (int j = threadIdx.x; j < p.G * 3; j += TPB) {
            const int g = j / 3, k = j % 3;
            float sum = 0.f;
            for (int b = 0; b < p.NB; b++) sum += p.loss_part[((size_t)g * p.NB + b) * 3 + k];
            p.loss[j] = sum * p.inv_R;
        }
}

size_t act_lds(int H, int D) {
    const int HP = pitch_h(H);
    return sizeof(float) * ((size_t)up4(TR * pitch_x(D)) + 2 * TR * HP + 2 * TR + 8 * TR) + sizeof(int) * (4 * TR + 2 * TR);
}

size_t rows_lds(int H, int D) {
    const int HP = pitch_h(H);
    return sizeof(float) * ((size_t)up4(TR * pitch_x(D)) + 8 * TR * HP + 15 * TR + 8 * TR) + sizeof(int) * TR;
}

}  // namespace

hipError_t launch_wide_act(const WideAct& p, hipStream_t st) {
    const dim3 grid((unsigned)((p.E + TR - 1) / TR), (unsigned)p.G);
    const size_t lds = act_lds(p.H, p.D);
    if (p.H == 32)
        hipLaunchKernelGGL(k_wide_act<32>, grid, dim3(TPB), lds, st, p);
    else if (p.H == 64)
        hipLaunchKernelGGL(k_wide_act<64>, grid, dim3(TPB), lds, st, p);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// rows -> split partials -> gradient tensors (three launches on one stream)
hipError_t launch_wide_grad(const WideRows& rows, const WideGrads& gp, const WideReduce& rp, hipStream_t st) {
    const int H = rows.H;
    if (H != 32 && H != 64) return hipErrorInvalidValue;
    const size_t l_rows = rows_lds(H, rows.D);
    const size_t l_outer = sizeof(float) * ((size_t)TR * H + (size_t)TPB * H);
    const size_t l_w3 = sizeof(float) * ((size_t)TR * pitch_h(H) + TR * kWideStats + 4 * 64 * (H + 1));
    const dim3 g_rows((unsigned)rows.NB, (unsigned)rows.G);
    const dim3 g_outer(5u, (unsigned)gp.RS, (unsigned)gp.G);
    const dim3 g_w3((unsigned)((gp.A + 63) / 64), (unsigned)gp.RS, (unsigned)gp.G);
    const long long n = (long long)rp.G * rp.off.o[kWideSegs];
    const dim3 g_red((unsigned)((n + TPB - 1) / TPB));
    if (H == 32) {
        hipLaunchKernelGGL(k_wide_rows<32>, g_rows, dim3(TPB), l_rows, st, rows);
        hipLaunchKernelGGL(k_wide_outer<32>, g_outer, dim3(TPB), l_outer, st, gp);
        hipLaunchKernelGGL(k_wide_w3<32>, g_w3, dim3(TPB), l_w3, st, gp);
    } else {
        hipLaunchKernelGGL(k_wide_rows<64>, g_rows, dim3(TPB), l_rows, st, rows);
        hipLaunchKernelGGL(k_wide_outer<64>, g_outer, dim3(TPB), l_outer, st, gp);
        hipLaunchKernelGGL(k_wide_w3<64>, g_w3, dim3(TPB), l_w3, st, gp);
    }
    hipLaunchKernelGGL(k_wide_reduce, g_red, dim3(TPB), 0, st, rp);
    return hipGetLastError();
}

}  // namespace ms
