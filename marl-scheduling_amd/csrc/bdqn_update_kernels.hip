// bdqn_update_kernels.hip — BranchingDQN.update_policy (BranchingDQNModules.py:125-164) on gfx950 for
// one role's minibatch: the three forwards (q(s), q(s'), target(s')), the double-DQN target averaged
// over the branches, the MSE loss broadcast over the branches, its backward through the dueling head
// and both ReLU layers, and the gradient clamp to [-1, 1]; the HIP Adam (ppo_kernels.hip k_adam)
// then steps the online net. The minibatch (B <= 128 rows) is one 128-row operand of every product;
// the matrix work is on MFMA tiles, the per-row work (argmax, target, loss) on one block per row:
//
//   k_bdqn_upd_l1      layer 1 of the three forwards, [128 x obs] x [obs x 128] in 128-wide K chunks
//                      (block = (chunk, forward)) on v_mfma_f32_16x16x32_bf16: the int8 inputs are
//                      exact in bf16 and W1 is split into three exact bf16 terms in registers, so
//                      every product is exact and only the f32 accumulation rounds
//   k_bdqn_upd_l2      the chunks' partial sums in chunk order, + b1, ReLU; layer 2, + b2, ReLU
//   k_bdqn_upd_heads   the advantage and value heads of the three forwards: [128 x 128] x [128 x
//                      (ac_dim n + 1)] on v_mfma_f32_16x16x4_f32 (exact f32 products)
//   k_bdqn_upd_target  one block per row: per branch q = v + adv - mean(adv), the first argmax of
//                      q(s'), the target's q there, the branch mean, r + max_next * gamma * mask, the
//                      row's squared errors, d loss / d q and from it the head outputs' gradient
//   k_bdqn_upd_dout2   d out2 = dQ x [Wa; wv] per chunk of 64 head rows (f32 MFMA), chunk partials
//   k_bdqn_upd_back1   the partials in chunk order, ReLU mask -> d pre2; W2^T d pre2, mask -> d pre1
//   k_bdqn_upd_wgrad   dW2, dWa, dwv = d^T a over the rows (f32 MFMA) and the biases, clamped; the loss
//   k_bdqn_upd_w1      dW1 = d pre1^T x (bf16 MFMA: d pre1 as three exact bf16 terms, x exact), db1
//
// Every sum runs in a fixed order (MFMA accumulation is deterministic), so a replay reproduces the
// gradient bit for bit. Products are exact f32 products, sums f32 as the reference's torch forward /
// autograd; the summation orders differ from torch's GEMMs, so results agree within f32 rounding
// (tests/test_bdqn_gpu.py against oracle/bdqn_ref.py and torch autograd).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "ms_bdqn.h"

namespace ms {

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

constexpr int kUpdK = 128;  // layer-1 K chunk

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 mfma_bf16(const u4v& a, const u4v& b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                   0);
}
__device__ __forceinline__ float trunc_bf16(float x) { return __uint_as_float(__float_as_uint(x) & 0xffff0000u); }
// two values exact in bf16 -> one dword (element 2t = low half)
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
    return (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
}
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
        hi[t] = pack2(h[0], h[1]);
        mid[t] = pack2(m[0], m[1]);
        lo[t] = pack2(l[0], l[1]);
    }
}
__device__ __forceinline__ uint32_t pack_i8(int a, int b) { return pack2((float)a, (float)b); }
__device__ __forceinline__ float clampg(float g, float c) { return g < -c ? -c : (g > c ? c : g); }  // NaN stays

// head row o of a net: the Mn advantage rows, then the value row; NULL past it
__device__ __forceinline__ const float* head_row(const BdqnNet& net, int o, int Mn) {
    return o < Mn ? net.wa + (size_t)o * kBH : (o == Mn ? net.wv : nullptr);
}
__device__ __forceinline__ float head_bias(const BdqnNet& net, int o, int Mn) {
    return o < Mn ? net.ba[o] : (o == Mn ? net.bv[0] : 0.f);
}

// torch.argmax's pick of two candidates (value, index): NaN wins, else the larger, ties to the smaller
// index; index INT_MAX = no candidate
__device__ __forceinline__ bool argmax_takes(float b1, int i1, float b2, int i2) {
    if (i2 == 0x7fffffff) return false;
    if (i1 == 0x7fffffff) return true;
    const bool n1 = b1 != b1, n2 = b2 != b2;
    if (n1 || n2) return n1 && n2 ? i2 < i1 : n2;
    return b2 > b1 || (b2 == b1 && i2 < i1);
}

__device__ __forceinline__ float wave_sum(float v) {  // a fixed xor tree: every lane gets the same sum
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) v += __shfl_xor(v, sh);
    return v;
}

}  // namespace

// ---- layer 1, forward f (0 = q(s), 1 = q(s'), 2 = target(s')), K chunk kc: P[f][kc][b][h].
//      Wave w: hidden 64 (w >> 1) .. +63 (A = W1 rows, 4 tiles), rows 64 (w & 1) .. +63 (B = x, 4 tiles)
__global__ void __launch_bounds__(256) k_bdqn_upd_l1(BdqnUpd p) {
    const int kc = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int D = p.q.obs, B = p.B;
    const int8_t* x = f == 0 ? p.xs : p.xn;
    const float* w1 = f == 2 ? p.t.w1 : p.q.w1;
    const int h0 = 64 * (w >> 1), b0 = 64 * (w & 1);
    const bool xvec = (p.ld & 7) == 0, wvec = (D & 3) == 0;
    constexpr int S = kUpdK / 32;
    const int ns = min(S, (D - kc * kUpdK + 31) / 32);  // k-steps of this chunk (uniform)
    // every load of the chunk is issued before the first MFMA (one memory round trip per block):
    // x as raw bytes (8 per lane per row tile and step), W1 as f32 (8 per lane per hidden tile and step)
    uint32_t xr[S][4][2];
    float wr[S][4][8];
#pragma unroll
    for (int s = 0; s < S; s++) {
        const int k = kc * kUpdK + 32 * s + 8 * g;  // this lane's 8 inputs k .. k + 7
#pragma unroll
        for (int bt = 0; bt < 4; bt++) {
            const int b = b0 + 16 * bt + i;
            xr[s][bt][0] = xr[s][bt][1] = 0u;
            if (s < ns && b < B) {
                if (xvec && k + 8 <= D) {
                    const uint2 u = *reinterpret_cast<const uint2*>(x + (size_t)b * p.ld + k);
                    xr[s][bt][0] = u.x;
                    xr[s][bt][1] = u.y;
                } else {
#pragma unroll
                    for (int e = 0; e < 8; e++)
                        if (k + e < D) xr[s][bt][e >> 2] |= (uint32_t)(uint8_t)x[(size_t)b * p.ld + k + e] << (8 * (e & 3));
                }
            }
        }
#pragma unroll
        for (int ht = 0; ht < 4; ht++) {
            const float* wp = w1 + (size_t)(h0 + 16 * ht + i) * D + k;
            if (s < ns && wvec && k + 8 <= D) {
                const f4 a0 = *reinterpret_cast<const f4*>(wp), a1 = *reinterpret_cast<const f4*>(wp + 4);
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    wr[s][ht][e] = a0[e];
                    wr[s][ht][4 + e] = a1[e];
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; e++) wr[s][ht][e] = (s < ns && k + e < D) ? wp[e] : 0.f;
            }
        }
    }
    f4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int c = 0; c < 4; c++) acc[a][c] = (f4){0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < S; s++) {
        if (s >= ns) break;
        u4v xb[4];
#pragma unroll
        for (int bt = 0; bt < 4; bt++)
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint32_t dw = xr[s][bt][t >> 1];
                const int sh = 16 * (t & 1);
                xb[bt][t] = pack_i8((int)(int8_t)(dw >> sh), (int)(int8_t)(dw >> (sh + 8)));
            }
#pragma unroll
        for (int ht = 0; ht < 4; ht++) {
            u4v a3[3];
            split8(wr[s][ht], a3[0], a3[1], a3[2]);
#pragma unroll
            for (int bt = 0; bt < 4; bt++)
#pragma unroll
                for (int t = 0; t < 3; t++) acc[ht][bt] = mfma_bf16(a3[t], xb[bt], acc[ht][bt]);
        }
    }
    // tile (ht, bt): lane (i, g) holds hidden h0 + 16 ht + 4 g + q of row b0 + 16 bt + i
    float* out = p.l1p + (size_t)(f * p.nK + kc) * 128 * 128;
#pragma unroll
    for (int ht = 0; ht < 4; ht++)
#pragma unroll
        for (int bt = 0; bt < 4; bt++)
            *reinterpret_cast<f4*>(out + (size_t)(b0 + 16 * bt + i) * 128 + h0 + 16 * ht + 4 * g) = acc[ht][bt];
}

// ---- 8 rows of forward f: layer 1 = the chunks' partials in chunk order + b1, ReLU; layer 2 (the
//      sum over the hidden units in order, as a dot product), + b2, ReLU. Thread (h, rh): rows 4 rh .. +3
__global__ void __launch_bounds__(256) k_bdqn_upd_l2(BdqnUpd p) {
    __shared__ __align__(16) float o1[8][128];
    const int rt = blockIdx.x, f = blockIdx.y, t = threadIdx.x, h = t & 127, rh = t >> 7;
    const int r0 = 8 * rt + 4 * rh;
    const BdqnNet& net = f == 2 ? p.t : p.q;
    const float* src = p.l1p + (size_t)f * p.nK * 128 * 128 + (size_t)r0 * 128 + h;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    int kc = 0;
    for (; kc + 4 <= p.nK; kc += 4) {  // 16 loads in flight, added in chunk order
        float v[4][4];
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int r = 0; r < 4; r++) v[u][r] = src[(size_t)(kc + u) * 128 * 128 + r * 128];
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int r = 0; r < 4; r++) s[r] += v[u][r];
    }
    for (; kc < p.nK; kc++)
#pragma unroll
        for (int r = 0; r < 4; r++) s[r] += src[(size_t)kc * 128 * 128 + r * 128];
    const float bh = net.b1[h];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const float v = s[r] + bh, o = v > 0.f ? v : 0.f;
        o1[4 * rh + r][h] = o;
        if (f == 0) p.out1[(size_t)(r0 + r) * 128 + h] = o;
    }
    __syncthreads();
    const float* w2 = net.w2 + (size_t)h * kBH;  // output unit j = h
#pragma unroll
    for (int r = 0; r < 4; r++) s[r] = 0.f;
#pragma unroll 8
    for (int k4 = 0; k4 < 32; k4++) {
        const f4 wv = *reinterpret_cast<const f4*>(w2 + 4 * k4);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const f4 ov = *reinterpret_cast<const f4*>(&o1[4 * rh + r][4 * k4]);
            s[r] = fmaf(wv.x, ov.x, s[r]);
            s[r] = fmaf(wv.y, ov.y, s[r]);
            s[r] = fmaf(wv.z, ov.z, s[r]);
            s[r] = fmaf(wv.w, ov.w, s[r]);
        }
    }
    const float b2 = net.b2[h];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const float v = s[r] + b2;
        p.out2[((size_t)f * 128 + r0 + r) * 128 + h] = v > 0.f ? v : 0.f;
    }
}

// ---- head rows 32 ot .. 32 ot + 31 of forward f for all 128 rows: Q[f][b][o] = out2[f][b] . Wh[o] + bias.
//      Wave w: rows 32 w .. +31 (A, 2 tiles), head rows (B, 2 tiles); MFMA k-slot (kk, q) of lane group g
//      is hidden unit 16 kk + 4 g + q (the same permutation on both operands)
__global__ void __launch_bounds__(256) k_bdqn_upd_heads(BdqnUpd p) {
    const int ot = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int Mn = p.q.ac_dim * p.q.n;
    const BdqnNet& net = f == 2 ? p.t : p.q;
    const float* ar[2];
    const float* wr[2];
#pragma unroll
    for (int bt = 0; bt < 2; bt++) ar[bt] = p.out2 + ((size_t)f * 128 + 32 * w + 16 * bt + i) * 128 + 4 * g;
#pragma unroll
    for (int c = 0; c < 2; c++) wr[c] = head_row(net, 32 * ot + 16 * c + i, Mn);
    f4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int c = 0; c < 2; c++) acc[a][c] = (f4){0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < 8; kk++) {
        f4 av[2], wv[2];
#pragma unroll
        for (int bt = 0; bt < 2; bt++) av[bt] = *reinterpret_cast<const f4*>(ar[bt] + 16 * kk);
#pragma unroll
        for (int c = 0; c < 2; c++) wv[c] = wr[c] ? *reinterpret_cast<const f4*>(wr[c] + 16 * kk + 4 * g) : (f4){0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int bt = 0; bt < 2; bt++)
#pragma unroll
                for (int c = 0; c < 2; c++) acc[bt][c] = mfma4(av[bt][q], wv[c][q], acc[bt][c]);
    }
    // lane (i, g) holds Q[row 32 w + 16 bt + 4 g + q][head row 32 ot + 16 c + i]
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const int o = 32 * ot + 16 * c + i;
        const float bias = head_bias(net, o, Mn);
#pragma unroll
        for (int bt = 0; bt < 2; bt++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int b = 32 * w + 16 * bt + 4 * g + q;
                p.q3[((size_t)f * 128 + b) * p.Mp + o] = wr[c] ? acc[bt][c][q] + bias : 0.f;
            }
    }
}

// ---- one block per row b: per branch m q = (v + adv) - mean(adv) (BranchingDQNModules.py:99), the first
//      argmax of q(s') (torch.argmax), the target's q there (:139-141), q(s) at the taken action (:135);
//      the branch mean (:142), expected = r + max_next * gamma * mask (:144), the MSE over [B, ac_dim]
//      and its gradient; then dQ[b] = d loss / d (advantages, value) of q(s)
__global__ void __launch_bounds__(256) k_bdqn_upd_target(BdqnUpd p) {
    extern __shared__ __align__(16) float sq[];  // [3][Mp] the row's head outputs
    __shared__ float tq[32], dcur[32], dvs;
    __shared__ int acts[32];
    const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int M = p.q.ac_dim, n = p.q.n, Mn = M * n, Mp = p.Mp;
    float* dq = p.dq + (size_t)b * Mp;
    if (b >= p.B) {  // rows past the batch add nothing to the weight gradients
        for (int o = t; o < Mp; o += 256) dq[o] = 0.f;
        if (t == 0) p.lossb[b] = 0.f;
        return;
    }
    for (int x = t; x < 3 * Mp; x += 256) {
        const int f = x / Mp, o = x - f * Mp;
        sq[x] = p.q3[((size_t)f * 128 + b) * Mp + o];
    }
    if (t < M) {
        const int a = p.act[(size_t)b * p.act_ld + t];
        acts[t] = a < 0 ? 0 : (a >= n ? n - 1 : a);  // in range for a trainer's actions; clamped for LDS safety
    }
    __syncthreads();
    const float v0 = sq[Mn], v1 = sq[Mp + Mn], v2 = sq[2 * Mp + Mn];
    const float inv_n = 1.0f / (float)n;
    for (int m = w; m < M; m += 4) {
        const float* a0 = sq + m * n;
        const float* a1 = a0 + Mp;
        const float* a2 = a1 + Mp;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f;
        for (int a = lane; a < n; a += 64) {
            s0 += a0[a];
            s1 += a1[a];
            s2 += a2[a];
        }
        const float mean0 = wave_sum(s0) * inv_n, mean1 = wave_sum(s1) * inv_n, mean2 = wave_sum(s2) * inv_n;
        float best = 0.f;
        int bi = 0x7fffffff;
        for (int a = lane; a < n; a += 64) {
            const float qa = (v1 + a1[a]) - mean1;
            if (argmax_takes(best, bi, qa, a)) {
                best = qa;
                bi = a;
            }
        }
#pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) {
            const float ob = __shfl_xor(best, sh);
            const int oi = __shfl_xor(bi, sh);
            if (argmax_takes(best, bi, ob, oi)) {
                best = ob;
                bi = oi;
            }
        }
        if (lane == 0) {
            tq[m] = (v2 + a2[bi]) - mean2;
            dcur[m] = (v0 + a0[acts[m]]) - mean0;  // current q for now
        }
    }
    __syncthreads();
    if (t == 0) {
        float s = 0.f;
        for (int m = 0; m < M; m++) s += tq[m];
        const float max_next = s / (float)M;
        const float expected = p.rew[b] + max_next * p.gamma * p.mask[b];
        const float scale = 2.f / (float)(p.B * M);
        float l = 0.f, dv = 0.f;
        for (int m = 0; m < M; m++) {
            const float e = expected - dcur[m];
            l += e * e;
            const float gm = -e * scale;  // d mean((expected - current)^2) / d current
            dcur[m] = gm;
            dv += gm;
        }
        p.lossb[b] = l;
        dvs = dv;  // d loss / d v: the sum over the branches of d q (value.unsqueeze(2) broadcast)
    }
    __syncthreads();
    // d adv[m][a] = d q[m][a] - (sum_a' d q[m][a']) / n (the - mean(adv) term, :99); then d v; zero past
    for (int o = t; o < Mp; o += 256) {
        float d = 0.f;
        if (o < Mn) {
            const int m = o / n, a = o - m * n;
            const float gm = dcur[m];
            d = (a == acts[m] ? gm : 0.f) - gm / (float)n;
        } else if (o == Mn) {
            d = dvs;
        }
        dq[o] = d;
    }
}

// ---- d out2 partial of head-row chunk c: part[c][b][h] = sum_{o in chunk} dQ[b][o] Wh[o][h].
//      Wave w: rows 32 w .. +31 (A = dQ, 2 tiles) x all 128 hidden (B = Wh from LDS, 8 tiles)
__global__ void __launch_bounds__(256) k_bdqn_upd_dout2(BdqnUpd p) {
    __shared__ __align__(16) float ws[64][kBPitch];
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int Mn = p.q.ac_dim * p.q.n;
    for (int x = tid; x < 64 * 32; x += 256) {
        const int r = x >> 5, h4 = x & 31;
        const float* src = head_row(p.q, 64 * c + r, Mn);
        *reinterpret_cast<f4*>(&ws[r][4 * h4]) = src ? *reinterpret_cast<const f4*>(src + 4 * h4) : (f4){0, 0, 0, 0};
    }
    __syncthreads();
    f4 acc[2][8];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int e = 0; e < 8; e++) acc[a][e] = (f4){0, 0, 0, 0};
    const float* dr[2];
#pragma unroll
    for (int bt = 0; bt < 2; bt++) dr[bt] = p.dq + (size_t)(32 * w + 16 * bt + i) * p.Mp + 64 * c + 4 * g;
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
        f4 av[2];
#pragma unroll
        for (int bt = 0; bt < 2; bt++) av[bt] = *reinterpret_cast<const f4*>(dr[bt] + 16 * kk);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float* wrow = ws[16 * kk + 4 * g + q];
#pragma unroll
            for (int ht = 0; ht < 8; ht++) {
                const float bv = wrow[16 * ht + i];
#pragma unroll
                for (int bt = 0; bt < 2; bt++) acc[bt][ht] = mfma4(av[bt][q], bv, acc[bt][ht]);
            }
        }
    }
    float* out = p.d2p + (size_t)c * 128 * 128;
#pragma unroll
    for (int bt = 0; bt < 2; bt++)
#pragma unroll
        for (int ht = 0; ht < 8; ht++)
#pragma unroll
            for (int q = 0; q < 4; q++) out[(size_t)(32 * w + 16 * bt + 4 * g + q) * 128 + 16 * ht + i] = acc[bt][ht][q];
}

// ---- 4 rows: d out2 = the chunk partials in chunk order, ReLU mask -> d pre2; d out1 = W2^T d pre2 (the
//      sum over the output units in order), mask -> d pre1. Rows past the batch: zero. Thread (h, rh): rows
//      4 blockIdx.x + 2 rh, + 1
__global__ void __launch_bounds__(256) k_bdqn_upd_back1(BdqnUpd p) {
    __shared__ float d2[4][128];
    const int t = threadIdx.x, h = t & 127, rh = t >> 7;
    const int r0 = 4 * blockIdx.x + 2 * rh;
    const int nC = p.Mp / 64;
    const float* src = p.d2p + (size_t)r0 * 128 + h;
    float s[2] = {0.f, 0.f};
    int c = 0;
    for (; c + 8 <= nC; c += 8) {  // 16 loads in flight, added in chunk order
        float v[8][2];
#pragma unroll
        for (int u = 0; u < 8; u++)
#pragma unroll
            for (int r = 0; r < 2; r++) v[u][r] = src[(size_t)(c + u) * 128 * 128 + r * 128];
#pragma unroll
        for (int u = 0; u < 8; u++)
#pragma unroll
            for (int r = 0; r < 2; r++) s[r] += v[u][r];
    }
    for (; c < nC; c++)
#pragma unroll
        for (int r = 0; r < 2; r++) s[r] += src[(size_t)c * 128 * 128 + r * 128];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int b = r0 + r;
        const float d = (b < p.B && p.out2[(size_t)b * 128 + h] > 0.f) ? s[r] : 0.f;
        p.dpre2[(size_t)b * 128 + h] = d;
        d2[2 * rh + r][h] = d;
    }
    __syncthreads();
    float u[2] = {0.f, 0.f};
#pragma unroll 16
    for (int j = 0; j < 128; j++) {
        const float wj = p.q.w2[(size_t)j * kBH + h];
#pragma unroll
        for (int r = 0; r < 2; r++) u[r] = fmaf(wj, d2[2 * rh + r][j], u[r]);
    }
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int b = r0 + r;
        p.dpre1[(size_t)b * 128 + h] = (b < p.B && p.out1[(size_t)b * 128 + h] > 0.f) ? u[r] : 0.f;
    }
}

// ---- weight gradients of rows 32 blockIdx.x .. +31 of [W2 (128 rows); Wa (Mn rows); wv]: dW[r][h] =
//      sum_b d[b][r] a[b][h] (d = d pre2 with a = out1, or dQ with a = out2 of q(s)), the bias sum_b d[b][r],
//      clamped; block 0 also the loss. d and a are staged in LDS (one round trip of 16-B loads); wave w:
//      the block's 32 rows (A, 2 tiles) x hidden 32 w .. +31 (B, 2 tiles)
constexpr int kWgDP = 36, kWgAP = 132;  // LDS pitches (floats)
__global__ void __launch_bounds__(256) k_bdqn_upd_wgrad(BdqnUpd p) {
    extern __shared__ __align__(16) float sm[];
    float* ds = sm;                  // [128][kWgDP]: d[b][r0 + 0..31]
    float* as = sm + 128 * kWgDP;    // [128][kWgAP]: a[b][h]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int Mn = p.q.ac_dim * p.q.n;
    const bool l2 = blockIdx.x < 4;
    const int r0 = l2 ? 32 * blockIdx.x : 32 * (blockIdx.x - 4);  // W2 row or head row
    const float* d = l2 ? p.dpre2 : p.dq;
    const int dld = l2 ? 128 : p.Mp;
    const float* a = l2 ? p.out1 : p.out2;
    {
        f4 dv[4], av[16];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int x = tid + 256 * u, b = x >> 3, c4 = x & 7;
            dv[u] = *reinterpret_cast<const f4*>(d + (size_t)b * dld + r0 + 4 * c4);
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int x = tid + 256 * u, b = x >> 5, c4 = x & 31;
            av[u] = *reinterpret_cast<const f4*>(a + (size_t)b * 128 + 4 * c4);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int x = tid + 256 * u, b = x >> 3, c4 = x & 7;
            *reinterpret_cast<f4*>(ds + b * kWgDP + 4 * c4) = dv[u];
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int x = tid + 256 * u, b = x >> 5, c4 = x & 31;
            *reinterpret_cast<f4*>(as + b * kWgAP + 4 * c4) = av[u];
        }
    }
    __syncthreads();
    f4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int c = 0; c < 2; c++) acc[x][c] = (f4){0, 0, 0, 0};
#pragma unroll 4
    for (int kk = 0; kk < 8; kk++) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int b = 16 * kk + 4 * g + q;
            float av[2], bv[2];
#pragma unroll
            for (int rt = 0; rt < 2; rt++) av[rt] = ds[b * kWgDP + 16 * rt + i];
#pragma unroll
            for (int ht = 0; ht < 2; ht++) bv[ht] = as[b * kWgAP + 32 * w + 16 * ht + i];
#pragma unroll
            for (int rt = 0; rt < 2; rt++)
#pragma unroll
                for (int ht = 0; ht < 2; ht++) acc[rt][ht] = mfma4(av[rt], bv[ht], acc[rt][ht]);
        }
    }
    const float cl = p.clip;
    // lane (i, g) holds dW[row r0 + 16 rt + 4 g + q][hidden 32 w + 16 ht + i]
#pragma unroll
    for (int rt = 0; rt < 2; rt++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int r = r0 + 16 * rt + 4 * g + q;
#pragma unroll
            for (int ht = 0; ht < 2; ht++) {
                const int h = 32 * w + 16 * ht + i;
                const float v = clampg(acc[rt][ht][q], cl);
                if (l2)
                    p.g.w2[(size_t)r * kBH + h] = v;
                else if (r < Mn)
                    p.g.wa[(size_t)r * kBH + h] = v;
                else if (r == Mn)
                    p.g.wv[h] = v;
            }
        }
    if (tid < 32) {
        const int r = r0 + tid;
        float s = 0.f;
        for (int b = 0; b < p.B; b++) s += ds[b * kWgDP + tid];
        s = clampg(s, cl);
        if (l2)
            p.g.b2[r] = s;
        else if (r < Mn)
            p.g.ba[r] = s;
        else if (r == Mn)
            p.g.bv[0] = s;
    }
    if (blockIdx.x == 0 && tid == 64) {
        float l = 0.f;
        for (int b = 0; b < p.B; b++) l += p.lossb[b];
        p.g.loss[0] = l / (float)(p.B * p.q.ac_dim);
    }
}

// ---- dW1[h][k] = sum_b d pre1[b][h] x[b][k] for inputs 64 blockIdx.x .. +63, db1 (block 0). d pre1 and the
//      x tile are staged in LDS (one round trip); wave w: hidden 32 w .. +31 (A = d pre1^T as three exact
//      bf16 terms, 2 tiles) x the 64 inputs (B = x, 4 tiles)
constexpr int kW1DP = 132;  // LDS pitch (floats) of the staged d pre1 rows
__global__ void __launch_bounds__(256) k_bdqn_upd_w1(BdqnUpd p) {
    extern __shared__ __align__(16) float sm[];
    float* dp = sm;                                                        // [128][kW1DP]
    uint32_t* xs = reinterpret_cast<uint32_t*>(sm + 128 * kW1DP);          // [128][16] dwords = 64 inputs
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int k0 = 64 * blockIdx.x, D = p.q.obs;
    {
        f4 dv[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int x = tid + 256 * u, b = x >> 5, c4 = x & 31;
            dv[u] = *reinterpret_cast<const f4*>(p.dpre1 + (size_t)b * 128 + 4 * c4);
        }
        uint32_t xv[8];
        const bool fast = (p.ld & 3) == 0 && k0 + 64 <= D;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int x = tid + 256 * u, b = x >> 4, c = x & 15;
            uint32_t v = 0;
            if (b < p.B) {
                const int8_t* src = p.xs + (size_t)b * p.ld + k0 + 4 * c;
                if (fast) {
                    v = *reinterpret_cast<const uint32_t*>(src);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        if (k0 + 4 * c + e < D) v |= (uint32_t)(uint8_t)src[e] << (8 * e);
                }
            }
            xv[u] = v;
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int x = tid + 256 * u, b = x >> 5, c4 = x & 31;
            *reinterpret_cast<f4*>(dp + b * kW1DP + 4 * c4) = dv[u];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) xs[tid + 256 * u] = xv[u];
    }
    __syncthreads();
    const uint8_t* xb8 = reinterpret_cast<const uint8_t*>(xs);  // [128][64] bytes
    f4 acc[2][4];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int c = 0; c < 4; c++) acc[x][c] = (f4){0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const int bb = 32 * s + 8 * g;  // this lane's 8 rows bb .. bb + 7
        u4v a3[2][3];
#pragma unroll
        for (int ht = 0; ht < 2; ht++) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; e++) v[e] = dp[(bb + e) * kW1DP + 32 * w + 16 * ht + i];
            split8(v, a3[ht][0], a3[ht][1], a3[ht][2]);
        }
#pragma unroll
        for (int kt = 0; kt < 4; kt++) {
            u4v xb;
#pragma unroll
            for (int t = 0; t < 4; t++)
                xb[t] = pack_i8((int8_t)xb8[(bb + 2 * t) * 64 + 16 * kt + i], (int8_t)xb8[(bb + 2 * t + 1) * 64 + 16 * kt + i]);
#pragma unroll
            for (int ht = 0; ht < 2; ht++)
#pragma unroll
                for (int t = 0; t < 3; t++) acc[ht][kt] = mfma_bf16(a3[ht][t], xb, acc[ht][kt]);
        }
    }
    const float cl = p.clip;
    // lane (i, g) holds dW1[hidden 32 w + 16 ht + 4 g + q][input k0 + 16 kt + i]
#pragma unroll
    for (int ht = 0; ht < 2; ht++)
#pragma unroll
        for (int kt = 0; kt < 4; kt++) {
            const int k = k0 + 16 * kt + i;
            if (k < D)
#pragma unroll
                for (int q = 0; q < 4; q++)
                    p.g.w1[(size_t)(32 * w + 16 * ht + 4 * g + q) * D + k] = clampg(acc[ht][kt][q], cl);
        }
    if (blockIdx.x == 0 && tid < 128) {
        float s = 0.f;
        for (int b = 0; b < p.B; b++) s += dp[b * kW1DP + tid];
        p.g.b1[tid] = clampg(s, cl);
    }
}

hipError_t launch_bdqn_update(const BdqnUpd& p, hipStream_t st) {
    if (p.Mp % 64 || p.Mp > kUpdMaxHeadRows || p.Mp < p.q.ac_dim * p.q.n + 1 || p.B < 1 || p.B > 128 ||
        p.q.ac_dim > 32)
        return hipErrorInvalidValue;
    hipError_t e;
#define MS_UPD_LAUNCH(K, GRID, LDS)                                      \
    hipLaunchKernelGGL(K, GRID, dim3(256), LDS, st, p);                  \
    if ((e = hipGetLastError()) != hipSuccess) return e;
    MS_UPD_LAUNCH(k_bdqn_upd_l1, dim3((unsigned)p.nK, 3), 0)
    MS_UPD_LAUNCH(k_bdqn_upd_l2, dim3(16, 3), 0)
    MS_UPD_LAUNCH(k_bdqn_upd_heads, dim3((unsigned)(p.Mp / 32), 3), 0)
    MS_UPD_LAUNCH(k_bdqn_upd_target, dim3(128), sizeof(float) * 3 * (size_t)p.Mp)
    MS_UPD_LAUNCH(k_bdqn_upd_dout2, dim3((unsigned)(p.Mp / 64)), 0)
    MS_UPD_LAUNCH(k_bdqn_upd_back1, dim3(32), 0)
    MS_UPD_LAUNCH(k_bdqn_upd_wgrad, dim3((unsigned)(4 + p.Mp / 32)), sizeof(float) * 128 * (kWgDP + kWgAP))
    MS_UPD_LAUNCH(k_bdqn_upd_w1, dim3((unsigned)((p.q.obs + 63) / 64)), sizeof(float) * 128 * (kW1DP + 16))
#undef MS_UPD_LAUNCH
    return hipSuccess;
}

}  // namespace ms
