// bdqn_update_kernels.hip — BranchingDQN.update_policy (BranchingDQNModules.py:125-164) on gfx950 for
// one role's minibatch: the three forwards (q(s), q(s'), target(s')), the double-DQN target averaged
// over the branches, the MSE loss broadcast over the branches, its backward through the dueling head
// and both ReLU layers, and the gradient clamp to [-1, 1]; the HIP Adam (ppo_kernels.hip k_adam)
// then steps the online net. Four launches instead of ~80 torch / hipBLASLt ones:
//
//   k_bdqn_upd_l1   layer 1 of the three forwards, [B x obs] x [obs x 128] in 128-wide K chunks
//                   (block = (chunk, forward)); exact partial sums per chunk, added in chunk order
//   k_bdqn_upd_row  one block per minibatch row: layer 1 sums + ReLU, layer 2, value and advantage
//                   heads of the three forwards; per branch q = v + adv - mean(adv), the first argmax
//                   of q(s'), the target net's q there, the branch mean, the expected value
//                   r + max_next * gamma * mask, the row's squared errors and d loss / d q; then the
//                   backward to the row's advantage / value / layer-2 / layer-1 pre-activation grads
//   k_bdqn_upd_wh   dW2, db2, dWa, dba, dwv, dbv as sums over the B rows (fixed order), clamped; the loss
//   k_bdqn_upd_w1   dW1, db1 the same way (block = 64 input columns)
//
// Every sum runs in a fixed order, so a replay reproduces the gradient bit for bit. Products and sums
// are f32 as the reference's torch forward / autograd; the summation orders differ from torch's GEMMs,
// so results agree within f32 rounding (tests/test_bdqn_gpu.py against oracle/bdqn_ref.py).
#include <hip/hip_runtime.h>

#include "ms_bdqn.h"

namespace ms {

constexpr int kUpdK = 128;    // layer-1 K chunk
constexpr int kUpdPitch = 132;

__device__ __forceinline__ float clampg(float g, float c) { return g < -c ? -c : (g > c ? c : g); }  // NaN stays

// forward f: 0 = q(s), 1 = q(s'), 2 = target(s')
__global__ void __launch_bounds__(256) k_bdqn_upd_l1(BdqnUpd p) {
    extern __shared__ __align__(16) float sm[];
    float* xs = sm;                       // [kUpdK][kUpdPitch]: x[b][k0 + kk] at xs[kk][b]
    float* ws = sm + kUpdK * kUpdPitch;   // [kUpdK][kUpdPitch]: W1[h][k0 + kk] at ws[kk][h]
    const int kc = blockIdx.x, f = blockIdx.y, t = threadIdx.x;
    const int k0 = kc * kUpdK, D = p.q.obs, B = p.B;
    const int8_t* x = f == 0 ? p.xs : p.xn;
    const float* w1 = f == 2 ? p.t.w1 : p.q.w1;
    for (int i = t; i < 128 * kUpdK; i += 256) {
        const int r = i / kUpdK, kk = i - r * kUpdK, k = k0 + kk;
        xs[kk * kUpdPitch + r] = (r < B && k < D) ? (float)x[(size_t)r * p.ld + k] : 0.f;
        ws[kk * kUpdPitch + r] = k < D ? w1[(size_t)r * D + k] : 0.f;
    }
    __syncthreads();
    const int ty = t >> 4, tx = t & 15;  // rows 8 ty .. 8 ty + 7, hidden 8 tx .. 8 tx + 7
    float acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) acc[i][j] = 0.f;
    for (int kk = 0; kk < kUpdK; kk++) {
        const float4 xa = *reinterpret_cast<const float4*>(xs + kk * kUpdPitch + 8 * ty);
        const float4 xb = *reinterpret_cast<const float4*>(xs + kk * kUpdPitch + 8 * ty + 4);
        const float4 wa = *reinterpret_cast<const float4*>(ws + kk * kUpdPitch + 8 * tx);
        const float4 wb = *reinterpret_cast<const float4*>(ws + kk * kUpdPitch + 8 * tx + 4);
        const float xv[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
        const float wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < 8; j++) acc[i][j] = fmaf(xv[i], wv[j], acc[i][j]);
    }
    float* out = p.l1p + ((size_t)(f * p.nK + kc) * 128) * 128;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        float4* o = reinterpret_cast<float4*>(out + (size_t)(8 * ty + i) * 128 + 8 * tx);
        o[0] = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
        o[1] = make_float4(acc[i][4], acc[i][5], acc[i][6], acc[i][7]);
    }
}

// dot of a 128-float weight row (global, 16-B aligned) with an LDS vector
__device__ __forceinline__ float dot128(const float* __restrict__ w, const float* v) {
    float s = 0.f;
#pragma unroll 8
    for (int h = 0; h < 128; h += 4) {
        const float4 a = *reinterpret_cast<const float4*>(w + h);
        s = fmaf(a.x, v[h], s);
        s = fmaf(a.y, v[h + 1], s);
        s = fmaf(a.z, v[h + 2], s);
        s = fmaf(a.w, v[h + 3], s);
    }
    return s;
}

__global__ void __launch_bounds__(256) k_bdqn_upd_row(BdqnUpd p) {
    extern __shared__ __align__(16) float sm[];
    const int M = p.q.ac_dim, n = p.q.n, Mn = M * n;
    float* pre1 = sm;             // [3][128]
    float* out1 = pre1 + 384;     // [3][128]
    float* pre2 = out1 + 384;     // [3][128]
    float* out2 = pre2 + 384;     // [3][128]
    float* val = out2 + 384;      // [4]: v of the three forwards
    float* red = val + 4;         // [2][128] partial sums of the backward
    float* dcur = red + 256;      // [32 + 4]: d loss / d q(s)[branch at its action]; [32]: loss of the row
    float* tq = dcur + 36;        // [32]: target(s')[branch][argmax of q(s')]
    float* adv = tq + 32;         // [3][Mn]
    const int b = blockIdx.x, t = threadIdx.x;
    // ---- layer 1: the chunks' partial sums in chunk order, + bias, ReLU
    for (int i = t; i < 384; i += 256) {
        const int f = i >> 7, h = i & 127;
        float s = 0.f;
        const float* src = p.l1p + ((size_t)f * p.nK * 128 + b) * 128 + h;
        for (int kc = 0; kc < p.nK; kc++) s += src[(size_t)kc * 128 * 128];
        s += (f == 2 ? p.t.b1 : p.q.b1)[h];
        pre1[i] = s;
        out1[i] = s > 0.f ? s : 0.f;
    }
    __syncthreads();
    // ---- layer 2: thread j < 128 the online row j for forwards 0 and 1, 128 + j the target's for 2
    {
        const int j = t & 127;
        if (t < 128) {
            const float* w = p.q.w2 + (size_t)j * 128;
            const float s0 = dot128(w, out1) + p.q.b2[j], s1 = dot128(w, out1 + 128) + p.q.b2[j];
            pre2[j] = s0;
            pre2[128 + j] = s1;
            out2[j] = s0 > 0.f ? s0 : 0.f;
            out2[128 + j] = s1 > 0.f ? s1 : 0.f;
        } else {
            const float s2 = dot128(p.t.w2 + (size_t)j * 128, out1 + 256) + p.t.b2[j];
            pre2[256 + j] = s2;
            out2[256 + j] = s2 > 0.f ? s2 : 0.f;
        }
    }
    __syncthreads();
    // ---- value and advantage heads: item i < Mn + 1 of the online net (forwards 0 and 1), then of
    //      the target (forward 2); head row Mn is the value head
    for (int i = t; i < 2 * (Mn + 1); i += 256) {
        const bool tg = i > Mn;
        const int o = tg ? i - (Mn + 1) : i;
        const BdqnNet& net = tg ? p.t : p.q;
        const float* w = o < Mn ? net.wa + (size_t)o * 128 : net.wv;
        const float bias = o < Mn ? net.ba[o] : net.bv[0];
        if (!tg) {
            const float s0 = dot128(w, out2) + bias, s1 = dot128(w, out2 + 128) + bias;
            if (o < Mn) {
                adv[o] = s0;
                adv[Mn + o] = s1;
            } else {
                val[0] = s0;
                val[1] = s1;
            }
        } else {
            const float s2 = dot128(w, out2 + 256) + bias;
            if (o < Mn)
                adv[2 * Mn + o] = s2;
            else
                val[2] = s2;
        }
    }
    __syncthreads();
    // ---- per branch m: q = v + adv - mean(adv) (BranchingDQNModules.py:99); the first argmax of
    //      q(s') (torch.argmax), the target's q there (:139-141), q(s) at the taken action (:135)
    if (t < M) {
        const int m = t;
        float mean[3];
#pragma unroll
        for (int f = 0; f < 3; f++) {
            float s = 0.f;
            for (int a = 0; a < n; a++) s += adv[f * Mn + m * n + a];
            mean[f] = s / (float)n;
        }
        int am = 0;
        float best = (val[1] + adv[Mn + m * n]) - mean[1];
        for (int a = 1; a < n; a++) {
            const float qa = (val[1] + adv[Mn + m * n + a]) - mean[1];
            if (qa > best || (qa != qa && best == best)) {  // torch.argmax: first maximum, NaN wins
                best = qa;
                am = a;
            }
        }
        tq[m] = (val[2] + adv[2 * Mn + m * n + am]) - mean[2];
        const int act = p.act[(size_t)b * p.act_ld + m];
        dcur[m] = (val[0] + adv[m * n + act]) - mean[0];  // current q for now
    }
    __syncthreads();
    if (t == 0) {
        // max_next_q_vals.mean(1) (:142), expected = r + max_next * 0.99 * mask (:144), MSE over [B, M]
        float s = 0.f;
        for (int m = 0; m < M; m++) s += tq[m];
        const float max_next = s / (float)M;
        const float expected = p.rew[b] + max_next * p.gamma * p.mask[b];
        const float scale = 2.f / (float)(p.B * M);
        float l = 0.f, dvs = 0.f;
        for (int m = 0; m < M; m++) {
            const float e = expected - dcur[m];
            l += e * e;
            const float g = -e * scale;  // d mean((expected - current)^2) / d current
            dcur[m] = g;
            dvs += g;
        }
        p.lossb[b] = l;
        val[3] = dvs;  // d loss / d v: the sum over the branches of d q (value.unsqueeze(2) broadcast)
        p.dv[b] = dvs;
    }
    __syncthreads();
    // ---- d adv[m][a] = d q[m][a] - (sum_a' d q[m][a']) / n (the - mean(adv) term, :99)
    float* dadv = adv;  // forward 0's advantages are no longer needed: reuse for the gradient
    for (int o = t; o < Mn; o += 256) {
        const int m = o / n, a = o - m * n;
        const int act = p.act[(size_t)b * p.act_ld + m];
        const float g = dcur[m];
        const float d = (a == act ? g : 0.f) - g / (float)n;
        dadv[o] = d;
        p.dadv[(size_t)b * Mn + o] = d;
    }
    __syncthreads();
    // ---- d out2[h] = wv[h] dv + sum_o Wa[o][h] dadv[o] (two halves of o, added in order), ReLU
    {
        const int h = t & 127, half = t >> 7;
        const int o0 = half ? (Mn + 1) / 2 : 0, o1 = half ? Mn : (Mn + 1) / 2;
        float s = half ? 0.f : p.q.wv[h] * val[3];
        for (int o = o0; o < o1; o++) s = fmaf(p.q.wa[(size_t)o * 128 + h], dadv[o], s);
        red[t] = s;
    }
    __syncthreads();
    if (t < 128) {
        const float d2 = pre2[t] > 0.f ? red[t] + red[128 + t] : 0.f;
        red[t] = d2;  // d pre2 of forward 0
        p.dpre2[(size_t)b * 128 + t] = d2;
        p.out1[(size_t)b * 128 + t] = out1[t];
        p.out2[(size_t)b * 128 + t] = out2[t];
    }
    __syncthreads();
    // ---- d out1[h] = sum_j W2[j][h] d pre2[j], ReLU
    if (t < 128) {
        float s = 0.f;
        for (int j = 0; j < 128; j++) s = fmaf(p.q.w2[(size_t)j * 128 + t], red[j], s);
        p.dpre1[(size_t)b * 128 + t] = pre1[t] > 0.f ? s : 0.f;
    }
}

// weight gradients of the head and layer 2: output row r of [W2 (128 rows); Wa (Mn rows); wv (1 row)],
// column h, summed over the B rows in order; then the biases and the loss (block 0)
__global__ void __launch_bounds__(256) k_bdqn_upd_wh(BdqnUpd p) {
    const int Mn = p.q.ac_dim * p.q.n, nr = 128 + Mn + 1;
    const int t = threadIdx.x, h = t & 127;
    const float c = p.clip;
    for (int rr = 0; rr < 4; rr++) {
        const int r = blockIdx.x * 8 + (t >> 7) * 4 + rr;
        if (r >= nr) break;
        float s = 0.f, sb = 0.f;
        for (int b = 0; b < p.B; b++) {
            float d;
            const float* a;
            if (r < 128) {
                d = p.dpre2[(size_t)b * 128 + r];
                a = p.out1 + (size_t)b * 128;
            } else if (r < 128 + Mn) {
                d = p.dadv[(size_t)b * Mn + (r - 128)];
                a = p.out2 + (size_t)b * 128;
            } else {
                d = p.dv[b];
                a = p.out2 + (size_t)b * 128;
            }
            s = fmaf(d, a[h], s);
            sb += d;
        }
        if (r < 128) {
            p.g.w2[(size_t)r * 128 + h] = clampg(s, c);
            if (h == 0) p.g.b2[r] = clampg(sb, c);
        } else if (r < 128 + Mn) {
            p.g.wa[(size_t)(r - 128) * 128 + h] = clampg(s, c);
            if (h == 0) p.g.ba[r - 128] = clampg(sb, c);
        } else {
            p.g.wv[h] = clampg(s, c);
            if (h == 0) p.g.bv[0] = clampg(sb, c);
        }
    }
    if (blockIdx.x == 0 && t == 0) {
        float l = 0.f;
        for (int b = 0; b < p.B; b++) l += p.lossb[b];
        p.g.loss[0] = l / (float)(p.B * p.q.ac_dim);
    }
}

// dW1[h][k] = sum_b d pre1[b][h] x[b][k], db1: block = 64 input columns, thread = (h, 32 columns)
__global__ void __launch_bounds__(256) k_bdqn_upd_w1(BdqnUpd p) {
    extern __shared__ __align__(16) float sm[];
    float (*xs)[64] = reinterpret_cast<float (*)[64]>(sm);             // [128 rows][64 columns]
    float (*dp)[128] = reinterpret_cast<float (*)[128]>(sm + 128 * 64);  // [128 rows][128 hidden]
    const int t = threadIdx.x, k0 = blockIdx.x * 64, D = p.q.obs;
    for (int i = t; i < 128 * 64; i += 256) {
        const int r = i >> 6, kk = i & 63;
        xs[r][kk] = (r < p.B && k0 + kk < D) ? (float)p.xs[(size_t)r * p.ld + k0 + kk] : 0.f;
    }
    for (int i = t; i < 128 * 128; i += 256) {
        const int r = i >> 7, h = i & 127;
        dp[r][h] = r < p.B ? p.dpre1[(size_t)r * 128 + h] : 0.f;
    }
    __syncthreads();
    const int h = t >> 1, kh = (t & 1) * 32;
    float acc[32];
#pragma unroll
    for (int i = 0; i < 32; i++) acc[i] = 0.f;
    for (int b = 0; b < p.B; b++) {
        const float d = dp[b][h];
#pragma unroll
        for (int i = 0; i < 32; i++) acc[i] = fmaf(d, xs[b][kh + i], acc[i]);
    }
    const float c = p.clip;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        const int k = k0 + kh + i;
        if (k < D) p.g.w1[(size_t)h * D + k] = clampg(acc[i], c);
    }
    if (blockIdx.x == 0 && t < 128) {
        float s = 0.f;
        for (int b = 0; b < p.B; b++) s += dp[b][t];
        p.g.b1[t] = clampg(s, c);
    }
}

hipError_t launch_bdqn_update(const BdqnUpd& p, hipStream_t st) {
    const int Mn = p.q.ac_dim * p.q.n;
    hipLaunchKernelGGL(k_bdqn_upd_l1, dim3((unsigned)p.nK, 3), dim3(256), sizeof(float) * 2 * kUpdK * kUpdPitch, st, p);
    hipError_t e;
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const size_t lds_row = sizeof(float) * (4 * 384 + 4 + 256 + 36 + 32 + 3 * Mn);
    hipLaunchKernelGGL(k_bdqn_upd_row, dim3((unsigned)p.B), dim3(256), lds_row, st, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_bdqn_upd_wh, dim3((unsigned)((128 + Mn + 1 + 7) / 8)), dim3(256), 0, st, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_bdqn_upd_w1, dim3((unsigned)((p.q.obs + 63) / 64)), dim3(256), sizeof(float) * 128 * 192, st, p);
    return hipGetLastError();
}

}  // namespace ms
