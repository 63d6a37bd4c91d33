// ppo_kernels.hip — fused PPO loss gradient for groups of 16-wide actor-critics on gfx950.
//
// One K-epoch step of PPO.update (PPOmodules.py:144-168) needs, per group g,
// d/dθ of  mean_r[ -min(ratio*adv, clamp(ratio)*adv) ] + 0.5*mean_r[(V-G)^2] - 0.01*mean_r[H]
// over R = T*E rows (torch Categorical semantics: probs renormalised,
// logits = log(clamp(p, eps, 1-eps)), entropy -sum(logits*p)). k_ppo_grad
// computes it in one pass over the int8 rollout buffer: for each 16-row tile a
// wave runs the actor and critic forward, the per-row loss derivatives and the
// backward pass on the f32 MFMA (v_mfma_f32_16x16x4_f32: an exact k-ordered
// fmaf chain), keeping the batch on the MFMA's column (lane) axis so that every
// layer's output feeds the next layer's B operand with no data movement (the
// A-operand weights are read with a permuted k order instead). The weight
// gradients are batch reductions, i.e. MFMAs with K = rows: their operands are
// the activations transposed through a small LDS tile, their accumulators stay
// in registers for the whole chunk. Each block writes one partial gradient
// vector; k_ppo_reduce sums the partials in a fixed order (deterministic) into
// the torch .grad tensors.
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/marlsched.h"
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
__device__ __forceinline__ float xsum4g(float v) {  // sum over lanes j, j+16, j+32, j+48
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}
__device__ __forceinline__ float xmax4g(float v) {
    v = fmaxf(v, __shfl_xor(v, 16));
    v = fmaxf(v, __shfl_xor(v, 32));
    return v;
}

// NQ = ceil(D/16) input tiles, NT = ceil(A/16) action tiles. One wave per block.
template <int NQ, int NT>
__global__ void __launch_bounds__(64) k_ppo_grad(PpoArgs p) {
    constexpr int TP = 17;  // transpose tile pitch (floats)
    constexpr int NTR = 7 + NT;
    const int lane = threadIdx.x;
    const int g4 = lane >> 4;  // MFMA k-group / C-row group
    const int j = lane & 15;   // batch row within the tile (C column)
    const int grp = blockIdx.x / p.n_chunks;
    const int chunk = blockIdx.x % p.n_chunks;
    const int D = p.D, A = p.A;
    const int D4 = (D + 3) & ~3;
    const int S1 = D4 / 4;
    const int u = p.unit_of_group[grp];

    extern __shared__ __align__(16) float sm[];
    float* sW1 = sm;                   // [16][D4]
    float* sC1 = sW1 + 16 * D4;        // [16][D4]
    float* sW2 = sC1 + 16 * D4;        // [16][16]
    float* sC2 = sW2 + 256;            // [16][16]
    float* sW3 = sC2 + 256;            // [16*NT][16] (zero rows >= A)
    float* sb1 = sW3 + 256 * NT;       // 16
    float* sb2 = sb1 + 16;             // 16
    float* sb3 = sb2 + 16;             // 16*NT
    float* sc3 = sb3 + 16 * NT;        // 16 (critic output row)
    float* scb1 = sc3 + 16;            // 16
    float* scb2 = scb1 + 16;           // 16
    float* scb3 = scb2 + 16;           // 1 (+3 pad)
    float* sT = scb3 + 4;              // [NTR][16][TP] transposes
    int8_t* sX = reinterpret_cast<int8_t*>(sT + NTR * 16 * TP);  // [16][stride]

    // ---- stage this group's weights
    {
        const float* W1 = p.w1 + (size_t)grp * 16 * D;
        const float* C1 = p.cw1 + (size_t)grp * 16 * D;
        for (int i = lane; i < 16 * D4; i += 64) {
            int r = i / D4, c = i % D4;
            sW1[i] = c < D ? W1[r * D + c] : 0.f;
            sC1[i] = c < D ? C1[r * D + c] : 0.f;
        }
        for (int i = lane; i < 256; i += 64) {
            sW2[i] = p.w2[(size_t)grp * 256 + i];
            sC2[i] = p.cw2[(size_t)grp * 256 + i];
        }
        for (int i = lane; i < 256 * NT; i += 64) {
            int a = i / 16;
            sW3[i] = a < A ? p.w3[((size_t)grp * A + a) * 16 + (i % 16)] : 0.f;
        }
        for (int i = lane; i < 16 * NT; i += 64) sb3[i] = i < A ? p.b3[(size_t)grp * A + i] : 0.f;
        if (lane < 16) {
            sb1[lane] = p.b1[grp * 16 + lane];
            sb2[lane] = p.b2[grp * 16 + lane];
            sc3[lane] = p.cw3[grp * 16 + lane];
            scb1[lane] = p.cb1[grp * 16 + lane];
            scb2[lane] = p.cb2[grp * 16 + lane];
        }
        if (lane == 0) scb3[0] = p.cb3[grp];
    }
    __syncthreads();

    f4 gW1[NQ], gC1[NQ], gW3[NT];
    f4 gW2 = {0, 0, 0, 0}, gC2 = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < NQ; q++) gW1[q] = gC1[q] = (f4){0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < NT; t++) gW3[t] = (f4){0, 0, 0, 0};
    float db1[4] = {0, 0, 0, 0}, db2[4] = {0, 0, 0, 0}, cdb1[4] = {0, 0, 0, 0}, cdb2[4] = {0, 0, 0, 0};
    float db3[NT][4];
#pragma unroll
    for (int t = 0; t < NT; t++) db3[t][0] = db3[t][1] = db3[t][2] = db3[t][3] = 0.f;
    float gC3[4] = {0, 0, 0, 0}, cdb3 = 0.f;
    float l_min = 0.f, l_mse = 0.f, l_ent = 0.f;
    const float eps = 1.1920928955078125e-07f;

    const int stride4 = p.stride >> 2;
    const int R = (int)p.R, E = (int)p.E;
    const int tile0 = chunk * p.chunk_tiles;
    const int tile_end = min(tile0 + p.chunk_tiles, (R + 15) >> 4);
    // lane (j, g4) copies dwords g4 + 4m of tile row j and owns row j's scalars; the next
    // tile's loads are issued before the current tile is processed (register prefetch)
    constexpr int kPreW = 16;  // 16 rows x 256 B / 64 lanes
    uint32_t pre[kPreW];
    int pre_act = 0;
    float pre_olp = 0.f, pre_G = 0.f;
    auto prefetch = [&](int tile) {
        const int r = tile * 16 + j;
        const bool ok = r < R;
        const size_t ru = (size_t)(ok ? r : 0) * p.U + u;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(p.states + ru * p.stride);
#pragma unroll
        for (int m = 0; m < kPreW; m++) {
            const int cc = g4 + 4 * m;
            pre[m] = (ok && cc < stride4) ? src[cc] : 0u;
        }
        pre_act = ok ? p.actions[ru] : 0;
        pre_olp = ok ? p.old_lp[ru] : 0.f;
        const int t = ok ? r / E : 0;
        pre_G = ok ? p.ret[((size_t)(r - t * E) * p.G + grp) * p.T + t] : 0.f;
    };
    if (tile0 < tile_end) prefetch(tile0);
    for (int tile = tile0; tile < tile_end; tile++) {
        // ---- stage the tile's 16 observation rows (int8) in LDS, then start the next tile's loads
#pragma unroll
        for (int m = 0; m < kPreW; m++) {
            const int cc = g4 + 4 * m;
            if (cc < stride4) reinterpret_cast<uint32_t*>(sX)[j * stride4 + cc] = pre[m];
        }
        const bool valid = tile * 16 + j < R;
        const int act = pre_act;
        const float olp = pre_olp, G = pre_G;
        if (tile + 1 < tile_end) prefetch(tile + 1);
        __syncthreads();

        // ---- forward, layer 1 (actor + critic share the X operand)
        f4 a1 = {0, 0, 0, 0}, c1 = {0, 0, 0, 0};
        for (int s = 0; s < S1; s++) {
            float x = (float)sX[j * p.stride + 4 * s + g4];
            a1 = mfma4(sW1[j * D4 + 4 * s + g4], x, a1);
            c1 = mfma4(sC1[j * D4 + 4 * s + g4], x, c1);
        }
        float h1[4], hc1[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            h1[q] = tanhf(a1[q] + sb1[4 * g4 + q]);
            hc1[q] = tanhf(c1[q] + scb1[4 * g4 + q]);
        }
        // layer 2: B operand = layer-1 output as is; A reads W2 with k permuted (k_true = 4*g4 + s)
        f4 a2 = {0, 0, 0, 0}, c2 = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 4; s++) {
            a2 = mfma4(sW2[j * 16 + 4 * g4 + s], h1[s], a2);
            c2 = mfma4(sC2[j * 16 + 4 * g4 + s], hc1[s], c2);
        }
        float h2[4], hc2[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            h2[q] = tanhf(a2[q] + sb2[4 * g4 + q]);
            hc2[q] = tanhf(c2[q] + scb2[4 * g4 + q]);
        }
        // actor layer 3 -> logits z[a = 16t + 4*g4 + q][row j]
        float z[NT][4];
#pragma unroll
        for (int t = 0; t < NT; t++) {
            f4 zz = {0, 0, 0, 0};
#pragma unroll
            for (int s = 0; s < 4; s++) zz = mfma4(sW3[(16 * t + j) * 16 + 4 * g4 + s], h2[s], zz);
#pragma unroll
            for (int q = 0; q < 4; q++) z[t][q] = zz[q] + sb3[16 * t + 4 * g4 + q];
        }
        // critic output V (one row of the last layer, summed across the 4 lane groups)
        float vp = 0.f;
#pragma unroll
        for (int q = 0; q < 4; q++) vp = fmaf(sc3[4 * g4 + q], hc2[q], vp);
        const float V = xsum4g(vp) + scb3[0];

        // ---- softmax (nn.Softmax) + Categorical(probs) renormalisation, log-prob, entropy
        float m = -INFINITY;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (16 * t + 4 * g4 + q < A) m = fmaxf(m, z[t][q]);
        m = xmax4g(m);
        float pe[NT][4], s0 = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                pe[t][q] = (16 * t + 4 * g4 + q < A) ? expf(z[t][q] - m) : 0.f;
                s0 += pe[t][q];
            }
        const float inv0 = 1.f / xsum4g(s0);
        float s1 = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                pe[t][q] *= inv0;  // softmax output (same arithmetic as k_act)
                s1 += pe[t][q];
            }
        const float inv1 = 1.f / xsum4g(s1);
        float pn[NT][4], cl[NT][4], lp = 0.f, ent = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                int a = 16 * t + 4 * g4 + q;
                pn[t][q] = pe[t][q] * inv1;
                float pc = fminf(fmaxf(pn[t][q], eps), 1.f - eps);
                cl[t][q] = logf(pc);
                if (a < A) {
                    if (a == act) lp += cl[t][q];
                    ent -= cl[t][q] * pn[t][q];
                }
            }
        lp = xsum4g(lp);
        ent = xsum4g(ent);

        // ---- per-row loss derivatives (loss.mean() over R rows)
        const float ratio = expf(lp - olp);
        const float adv = G - V;
        const float sur1 = ratio * adv;
        const float rc = fminf(fmaxf(ratio, 1.f - p.eps_clip), 1.f + p.eps_clip);
        const float sur2 = rc * adv;
        const float inr = (ratio >= 1.f - p.eps_clip && ratio <= 1.f + p.eps_clip) ? 1.f : 0.f;
        float dmin;  // d min(s1, s2) / d ratio (torch.minimum splits ties)
        if (sur1 < sur2)
            dmin = adv;
        else if (sur2 < sur1)
            dmin = adv * inr;
        else
            dmin = 0.5f * adv + 0.5f * adv * inr;
        const float w = valid ? p.inv_R : 0.f;
        const float g_lp = -dmin * w * ratio;  // d loss / d logp (exp backward uses the result)
        const float g_v = (V - G) * w;         // 0.5 * d MSE / d V
        const float g_h = -0.01f * w;          // d loss / d entropy
        if (valid && g4 == 0) {
            l_min += -fminf(sur1, sur2);
            l_mse += (V - G) * (V - G);
            l_ent += ent;
        }
        // d loss / d pn  -> d / d p (renormalisation) -> d / d z (softmax)
        float dpn[NT][4], x1 = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                int a = 16 * t + 4 * g4 + q;
                float v = 0.f;
                if (a < A) {
                    float dc = (a == act ? g_lp : 0.f) - g_h * pn[t][q];
                    float in = (pn[t][q] >= eps && pn[t][q] <= 1.f - eps) ? 1.f : 0.f;
                    v = dc * in * __builtin_amdgcn_rcpf(fminf(fmaxf(pn[t][q], eps), 1.f - eps)) - g_h * cl[t][q];
                }
                dpn[t][q] = v;
                x1 += v * pe[t][q];
            }
        x1 = xsum4g(x1);
        float gz[NT][4], x2 = 0.f;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                float dp = (dpn[t][q] - x1 * inv1) * inv1;
                gz[t][q] = dp;
                x2 += dp * pe[t][q];
            }
        x2 = xsum4g(x2);
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) gz[t][q] = pe[t][q] * (gz[t][q] - x2);

        // ---- backward through the hidden layers (same no-movement trick, transposed weights)
        f4 d2 = {0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int s = 0; s < 4; s++) d2 = mfma4(sW3[(16 * t + 4 * g4 + s) * 16 + j], gz[t][s], d2);
        float dl2[4], dc2[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            dl2[q] = d2[q] * (1.f - h2[q] * h2[q]);
            dc2[q] = sc3[4 * g4 + q] * g_v * (1.f - hc2[q] * hc2[q]);
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
            dl1[q] = d1[q] * (1.f - h1[q] * h1[q]);
            dc1[q] = e1[q] * (1.f - hc1[q] * hc1[q]);
        }
        // bias gradients and the critic output layer (VALU; reduced over rows at the end)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            db1[q] += dl1[q];
            db2[q] += dl2[q];
            cdb1[q] += dc1[q];
            cdb2[q] += dc2[q];
            gC3[q] = fmaf(g_v, hc2[q], gC3[q]);
#pragma unroll
            for (int t = 0; t < NT; t++) db3[t][q] += gz[t][q];
        }
        if (g4 == 0) cdb3 += g_v;

        // ---- weight gradients: batch reductions as MFMAs with K = rows (operands transposed via LDS)
        float* T_d1 = sT;
        float* T_d2 = sT + 1 * 16 * TP;
        float* T_h1 = sT + 2 * 16 * TP;
        float* T_h2 = sT + 3 * 16 * TP;
        float* T_e1 = sT + 4 * 16 * TP;
        float* T_e2 = sT + 5 * 16 * TP;
        float* T_k1 = sT + 6 * 16 * TP;
        float* T_gz = sT + 7 * 16 * TP;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int f = 4 * g4 + q;
            T_d1[f * TP + j] = dl1[q];
            T_d2[f * TP + j] = dl2[q];
            T_h1[f * TP + j] = h1[q];
            T_h2[f * TP + j] = h2[q];
            T_e1[f * TP + j] = dc1[q];
            T_e2[f * TP + j] = dc2[q];
            T_k1[f * TP + j] = hc1[q];
#pragma unroll
            for (int t = 0; t < NT; t++) T_gz[(t * 16 + f) * TP + j] = gz[t][q];
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const int rr = 4 * s + g4;  // tile row supplied by this lane at k-step s
            const float ad1 = T_d1[j * TP + rr];
            const float ae1 = T_e1[j * TP + rr];
#pragma unroll
            for (int q = 0; q < NQ; q++) {
                int d = 16 * q + j;
                float xv = d < D ? (float)sX[rr * p.stride + d] : 0.f;
                gW1[q] = mfma4(ad1, xv, gW1[q]);
                gC1[q] = mfma4(ae1, xv, gC1[q]);
            }
            gW2 = mfma4(T_d2[j * TP + rr], T_h1[j * TP + rr], gW2);
            gC2 = mfma4(T_e2[j * TP + rr], T_k1[j * TP + rr], gC2);
            const float bh2 = T_h2[j * TP + rr];
#pragma unroll
            for (int t = 0; t < NT; t++) gW3[t] = mfma4(T_gz[(t * 16 + j) * TP + rr], bh2, gW3[t]);
        }
        __syncthreads();
    }

    // ---- write this block's partial gradient vector
    const POff o = poff(D, A);
    float* out = p.partials + ((size_t)grp * p.n_chunks + chunk) * p.P;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int f = 4 * g4 + q;  // C row (output feature) held in register q
#pragma unroll
        for (int qq = 0; qq < NQ; qq++) {
            int d = 16 * qq + j;
            if (d < D) {
                out[o.w1 + f * D + d] = gW1[qq][q];
                out[o.cw1 + f * D + d] = gC1[qq][q];
            }
        }
        out[o.w2 + f * 16 + j] = gW2[q];
        out[o.cw2 + f * 16 + j] = gC2[q];
#pragma unroll
        for (int t = 0; t < NT; t++) {
            int a = 16 * t + f;
            if (a < A) out[o.w3 + a * 16 + j] = gW3[t][q];
        }
        float v;
        v = xsum16(db1[q]);
        if (j == 0) out[o.b1 + f] = v;
        v = xsum16(db2[q]);
        if (j == 0) out[o.b2 + f] = v;
        v = xsum16(cdb1[q]);
        if (j == 0) out[o.cb1 + f] = v;
        v = xsum16(cdb2[q]);
        if (j == 0) out[o.cb2 + f] = v;
        v = xsum16(gC3[q]);
        if (j == 0) out[o.cw3 + f] = v;
#pragma unroll
        for (int t = 0; t < NT; t++) {
            v = xsum16(db3[t][q]);
            if (j == 0 && 16 * t + f < A) out[o.b3 + 16 * t + f] = v;
        }
    }
    float v = xsum16(cdb3);
    if (lane == 0) out[o.cb3] = v;
    v = xsum16(l_min);
    if (lane == 0) out[o.loss + 0] = v * p.inv_R;
    v = xsum16(l_mse);
    if (lane == 0) out[o.loss + 1] = v * p.inv_R;
    v = xsum16(l_ent);
    if (lane == 0) out[o.loss + 2] = v * p.inv_R;
}

// Sum the partials of every chunk (fixed order) and scatter into the .grad tensors.
__global__ void __launch_bounds__(256) k_ppo_reduce(const float* __restrict__ partials, int G, int n_chunks, int P,
                                                    int D, int A, GradOut go) {
    const int grp = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float* src = partials + (size_t)grp * n_chunks * P + i;
    float s = 0.f;
    for (int c = 0; c < n_chunks; c++) s += src[(size_t)c * P];
    const POff o = poff(D, A);
    float* dst;
    int k;
    if (i < o.b1) { dst = go.w1; k = 16 * D; }
    else if (i < o.w2) { dst = go.b1; k = 16; }
    else if (i < o.b2) { dst = go.w2; k = 256; }
    else if (i < o.w3) { dst = go.b2; k = 16; }
    else if (i < o.b3) { dst = go.w3; k = 16 * A; }
    else if (i < o.cw1) { dst = go.b3; k = A; }
    else if (i < o.cb1) { dst = go.cw1; k = 16 * D; }
    else if (i < o.cw2) { dst = go.cb1; k = 16; }
    else if (i < o.cb2) { dst = go.cw2; k = 256; }
    else if (i < o.cw3) { dst = go.cb2; k = 16; }
    else if (i < o.cb3) { dst = go.cw3; k = 16; }
    else if (i < o.loss) { dst = go.cb3; k = 1; }
    else { dst = go.loss; k = 3; }
    int base;
    if (dst == go.w1) base = o.w1; else if (dst == go.b1) base = o.b1; else if (dst == go.w2) base = o.w2;
    else if (dst == go.b2) base = o.b2; else if (dst == go.w3) base = o.w3; else if (dst == go.b3) base = o.b3;
    else if (dst == go.cw1) base = o.cw1; else if (dst == go.cb1) base = o.cb1; else if (dst == go.cw2) base = o.cw2;
    else if (dst == go.cb2) base = o.cb2; else if (dst == go.cw3) base = o.cw3; else if (dst == go.cb3) base = o.cb3;
    else base = o.loss;
    if (dst) dst[(size_t)grp * k + (i - base)] = s;
}

template <int NQ, int NT>
static hipError_t launch_grad_t(const PpoArgs& a, hipStream_t st) {
    const int D4 = (a.D + 3) & ~3;
    size_t lds = sizeof(float) * (2 * 16 * D4 + 2 * 256 + 256 * NT + 16 * 2 + 16 * NT + 16 * 3 + 4 + (7 + NT) * 16 * 17) +
                 16 * (size_t)a.stride;
    hipLaunchKernelGGL((k_ppo_grad<NQ, NT>), dim3((unsigned)(a.G * a.n_chunks)), dim3(64), lds, st, a);
    return hipGetLastError();
}

hipError_t launch_ppo_grad(const PpoArgs& a, const GradOut& go, hipStream_t st) {
    const int nq = (a.D + 15) / 16, nt = (a.A + 15) / 16;
    hipError_t e;
#define MS_PPO_CASE(Q, T)                                       \
    if (nq <= Q && nt <= T) {                                   \
        e = launch_grad_t<Q, T>(a, st);                         \
        goto reduce;                                            \
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
        hipLaunchKernelGGL(k_ppo_reduce, dim3((P + 255) / 256, a.G), dim3(256), 0, st, a.partials, a.G, a.n_chunks, P,
                           a.D, a.A, go);
    }
    return hipGetLastError();
}

int ppo_param_count(int D, int A) { return poff(D, A).total; }

}  // namespace ms
