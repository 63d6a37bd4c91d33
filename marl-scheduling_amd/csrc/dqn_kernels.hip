// dqn_kernels.hip — the DQN units of the reference (DQNmodules.py) batched over groups and env replicas.
//
// DQNEntity (DQNmodules.py:34-76) is nn.Sequential(Linear(D, 16), Tanh, Linear(16, A)); its
// selectAction takes the argmax of the Q-values (first maximum, torch.max) unless an
// epsilon draw explores. optimize_model (DQNmodules.py:97-154) regresses Q(s, a) on
// r + gamma * max_a' Q_target(s', a') with SmoothL1 (beta 1), clamps every gradient element
// to [-1, 1] and steps Adam. Here G nets of one unit type (one per unit for the divided agents,
// DividedFixPriceDQNAgent Agent.py:303-356) act on and learn from the rows of all E replicas:
//
//   k_dqn_act     one thread per (replica, unit) row: both layers from LDS-resident weights, the
//                 argmax, the epsilon decision on a given or Philox uniform;
//   k_dqn_grad    one thread per sampled transition: gather from the replay memory, policy and
//                 target forwards, the SmoothL1 derivative, the backward to dpre / dq; then the
//                 block sums its rows' weight gradients in a fixed order (deterministic) into one
//                 partial vector;
//   k_dqn_reduce  sums the partials in block order, clamps (p.grad.data.clamp_(-1, 1)) and writes
//                 torch .grad layouts; Adam is ms_adam_step.
//
// Rows per group are few hundred thousand at most and each costs ~2*16*(D + A) flop: these
// kernels are latency/VALU bound and small next to the env step; no MFMA tile fits a 16-wide
// layer of one row.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "ms_dqn.h"

namespace ms {

namespace {

__device__ __forceinline__ uint32_t mulhilo_d(uint32_t a, uint32_t b, uint32_t& hi) {
    const uint64_t p = (uint64_t)a * b;
    hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}

// Philox4x32-10 (Salmon et al., SC'11): four output words
__device__ __forceinline__ void philox4(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                        uint32_t (&o)[4]) {
    for (int r = 0; r < 10; r++) {
        uint32_t hi0, hi1;
        const uint32_t lo0 = mulhilo_d(0xD2511F53u, c0, hi0);
        const uint32_t lo1 = mulhilo_d(0xCD9E8D57u, c2, hi1);
        const uint32_t n0 = hi1 ^ c1 ^ k0;
        const uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    o[0] = c0;
    o[1] = c1;
    o[2] = c2;
    o[3] = c3;
}

// 53-bit double in [0, 1) from two words, random.random()'s construction
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// weights of one group, staged in LDS: W1 [H][D], b1 [H], W2 [A][H], b2 [A]
struct QW {
    const float *w1, *b1, *w2, *b2;
};

__device__ __forceinline__ QW stage_qnet(const QArgs& q, int g, float* s, int tid, int nthr) {
    const int D = q.D, A = q.A;
    const float* w1 = q.w1 + (int64_t)g * kQH * D;
    const float* b1 = q.b1 + (int64_t)g * kQH;
    const float* w2 = q.w2 + (int64_t)g * A * kQH;
    const float* b2 = q.b2 + (int64_t)g * A;
    float* s_w1 = s;
    float* s_b1 = s_w1 + kQH * D;
    float* s_w2 = s_b1 + kQH;
    float* s_b2 = s_w2 + A * kQH;
    for (int i = tid; i < kQH * D; i += nthr) s_w1[i] = w1[i];
    for (int i = tid; i < kQH; i += nthr) s_b1[i] = b1[i];
    for (int i = tid; i < A * kQH; i += nthr) s_w2[i] = w2[i];
    for (int i = tid; i < A; i += nthr) s_b2[i] = b2[i];
    return QW{s_w1, s_b1, s_w2, s_b2};
}

// hidden layer h = tanh(W1 x + b1) of one int8 row (dword loads; bytes past D meet no weight)
__device__ __forceinline__ void hidden_of(const QW& w, const int8_t* row, int D, float (&h)[kQH]) {
#pragma unroll
    for (int j = 0; j < kQH; j++) h[j] = 0.f;
    const uint32_t* r4 = reinterpret_cast<const uint32_t*>(row);
    for (int k4 = 0; 4 * k4 < D; k4++) {
        const uint32_t v = r4[k4];
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int k = 4 * k4 + b;
            if (k < D) {
                const float x = (float)(int8_t)(v >> (8 * b));
#pragma unroll
                for (int j = 0; j < kQH; j++) h[j] = fmaf(w.w1[j * D + k], x, h[j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kQH; j++) h[j] = tanhf(h[j] + w.b1[j]);
}

__device__ __forceinline__ float q_of(const QW& w, const float (&h)[kQH], int a) {
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < kQH; j++) q = fmaf(w.w2[a * kQH + j], h[j], q);
    return q + w.b2[a];
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// selectAction (DQNmodules.py:56-70) for rows obs[e][u][stride], unit u in group u / upg
__global__ void __launch_bounds__(256) k_dqn_act(DqnActArgs a) {
    extern __shared__ __align__(16) float s_act[];
    const int u = blockIdx.y;
    const int g = u / a.q.upg;
    const QW w = stage_qnet(a.q, g, s_act, threadIdx.x, blockDim.x);
    __syncthreads();
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.E) return;
    const int64_t row = e * a.U + u;
    float h[kQH];
    hidden_of(w, a.obs + row * a.stride, a.q.D, h);
    int best = 0;
    float bq = q_of(w, h, 0);
    for (int i = 1; i < a.q.A; i++) {  // torch.max: the first maximal index
        const float qi = q_of(w, h, i);
        if (qi > bq) {
            bq = qi;
            best = i;
        }
    }
    double u1, u2;
    if (a.uniforms) {
        u1 = a.uniforms[row];
        u2 = a.uniforms[a.E * a.U + row];
    } else {
        const uint64_t off = a.offset + (a.offset_dev ? *a.offset_dev : 0ull);
        uint32_t o[4];
        philox4((uint32_t)row, (uint32_t)(row >> 32), (uint32_t)off, (uint32_t)(off >> 32), (uint32_t)a.seed,
                (uint32_t)(a.seed >> 32), o);
        u1 = u53(o[0], o[1]);
        u2 = u53(o[2], o[3]);
    }
    // sample > eps_treshold -> greedy, else random.randrange(numberOfActions)
    int act = best;
    if (!(u1 > a.eps)) {
        act = (int)(u2 * a.q.A);
        if (act >= a.q.A) act = a.q.A - 1;
    }
    a.action[row] = (int8_t)act;
    if (a.greedy) a.greedy[row] = (int8_t)best;
}

// ---------------------------------------------------------------------------------------------
// optimize_model (DQNmodules.py:97-154): one thread per sampled transition of group g
__global__ void __launch_bounds__(256) k_dqn_grad(DqnGradArgs a) {
    extern __shared__ __align__(16) float s_grad[];
    const int g = blockIdx.y, tid = threadIdx.x;
    const int D = a.q.D, A = a.q.A;
    const int wfl = kQH * D + kQH + A * kQH + A;
    const QW wp = stage_qnet(a.q, g, s_grad, tid, blockDim.x);
    const QW wt = stage_qnet(a.t, g, s_grad + wfl, tid, blockDim.x);
    float* s_dpre = s_grad + 2 * wfl;          // [256][kQH + 1]
    float* s_h = s_dpre + 256 * (kQH + 1);     // [256][kQH + 1]
    float* s_gd = s_h + 256 * (kQH + 1);       // [256]
    float* s_loss = s_gd + 256;                // [256]
    int* s_a = reinterpret_cast<int*>(s_loss + 256);           // [256]
    int8_t* s_x = reinterpret_cast<int8_t*>(s_a + 256);        // [256][xp]
    const int xp = a.xpitch;
    __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * 256 + tid;  // row within the group
    float gd = 0.f, lossv = 0.f;
    int act = 0;
    float h[kQH];
#pragma unroll
    for (int j = 0; j < kQH; j++) h[j] = 0.f;
    if (r < a.rows) {
        // row r = ((e * upg) + j) * B + b
        const int64_t eb = r / a.B;
        const int b = (int)(r - eb * a.B);
        const int64_t e = eb / a.q.upg;
        const int ju = (int)(eb - e * a.q.upg);
        const int u = g * a.q.upg + ju;
        const int64_t eu = e * a.U + u;
        const int idx = a.samples[eu * a.B + b];
        const int64_t m = eu * a.cap + idx;
        const int8_t* xs = a.states + m * a.stride;
        const uint32_t* x4 = reinterpret_cast<const uint32_t*>(xs);
        uint32_t* dx = reinterpret_cast<uint32_t*>(s_x + tid * xp);
        for (int k4 = 0; 4 * k4 < D; k4++) dx[k4] = x4[k4];
        hidden_of(wp, xs, D, h);
        act = a.actions[m];
        const float q_sa = q_of(wp, h, act);  // policy_net(state).gather(1, action)
        float ht[kQH];
        hidden_of(wt, a.next_states + m * a.stride, D, ht);
        float qmax = q_of(wt, ht, 0);  // target_net(next_state).max(1)[0]
        for (int i = 1; i < A; i++) qmax = fmaxf(qmax, q_of(wt, ht, i));
        // expected = next_state_values * GAMMA + reward (float32 ops, as torch)
        const float y = __fadd_rn(__fmul_rn(qmax, a.gamma), a.rewards[m]);
        const float d = q_sa - y;
        const float ad = fabsf(d);
        lossv = ad < 1.f ? 0.5f * d * d : ad - 0.5f;  // SmoothL1Loss (beta = 1), mean over the rows
        gd = (ad < 1.f ? d : (d > 0.f ? 1.f : -1.f)) * a.inv_rows;
    }
    // backward of the taken action's Q: dq = gd at `act`
#pragma unroll
    for (int j = 0; j < kQH; j++) {
        const float dh = gd * wp.w2[act * kQH + j];
        s_dpre[tid * (kQH + 1) + j] = dh * (1.f - h[j] * h[j]);
        s_h[tid * (kQH + 1) + j] = h[j];
    }
    s_gd[tid] = gd;
    s_loss[tid] = lossv;
    s_a[tid] = r < a.rows ? act : -1;
    __syncthreads();
    // the block's weight gradients, each a fixed-order sum over its rows
    const int nrow = (int)min((int64_t)256, a.rows - (int64_t)blockIdx.x * 256);
    float* out = a.partials + ((int64_t)g * gridDim.x + blockIdx.x) * a.P;
    for (int o = tid; o < kQH * D; o += 256) {  // dW1[j][k] = sum_r dpre[r][j] * x[r][k]
        const int j = o / D, k = o - j * D;
        float s = 0.f;
        for (int rr = 0; rr < nrow; rr++) s = fmaf(s_dpre[rr * (kQH + 1) + j], (float)s_x[rr * xp + k], s);
        out[o] = s;
    }
    for (int o = tid; o < kQH; o += 256) {  // db1
        float s = 0.f;
        for (int rr = 0; rr < nrow; rr++) s += s_dpre[rr * (kQH + 1) + o];
        out[kQH * D + o] = s;
    }
    for (int o = tid; o < A * kQH; o += 256) {  // dW2[i][j] = sum_{r: a_r = i} gd_r * h_r[j]
        const int i = o / kQH, j = o - i * kQH;
        float s = 0.f;
        for (int rr = 0; rr < nrow; rr++)
            if (s_a[rr] == i) s = fmaf(s_gd[rr], s_h[rr * (kQH + 1) + j], s);
        out[kQH * D + kQH + o] = s;
    }
    for (int o = tid; o < A; o += 256) {  // db2
        float s = 0.f;
        for (int rr = 0; rr < nrow; rr++)
            if (s_a[rr] == o) s += s_gd[rr];
        out[kQH * D + kQH + A * kQH + o] = s;
    }
    if (tid == 0) {
        float s = 0.f;
        for (int rr = 0; rr < nrow; rr++) s += s_loss[rr];
        out[wfl] = s;
    }
}

// partials [G][nblk][P] -> clamped gradients (torch layouts) and the loss per group
__global__ void __launch_bounds__(256) k_dqn_reduce(DqnReduceArgs a) {
    const int g = blockIdx.y;
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= a.P) return;
    const float* src = a.partials + (int64_t)g * a.nblk * a.P + p;
    float s = 0.f;
    for (int b = 0; b < a.nblk; b++) s += src[(int64_t)b * a.P];
    const int D = a.D, A = a.A;
    const int o_b1 = kQH * D, o_w2 = o_b1 + kQH, o_b2 = o_w2 + A * kQH, o_loss = o_b2 + A;
    if (p == o_loss) {
        a.loss[g] = s * a.inv_rows;
        return;
    }
    if (a.clip > 0.f) s = fminf(fmaxf(s, -a.clip), a.clip);
    if (p < o_b1)
        a.w1[(int64_t)g * kQH * D + p] = s;
    else if (p < o_w2)
        a.b1[(int64_t)g * kQH + p - o_b1] = s;
    else if (p < o_b2)
        a.w2[(int64_t)g * A * kQH + p - o_w2] = s;
    else
        a.b2[(int64_t)g * A + p - o_b2] = s;
}

size_t dqn_act_lds(const QArgs& q) { return sizeof(float) * (size_t)(kQH * q.D + kQH + q.A * kQH + q.A); }

size_t dqn_grad_lds(const QArgs& q, int xpitch) {
    const size_t wfl = (size_t)(kQH * q.D + kQH + q.A * kQH + q.A);
    return sizeof(float) * (2 * wfl + 2 * 256 * (kQH + 1) + 2 * 256) + sizeof(int) * 256 + (size_t)256 * xpitch;
}

hipError_t launch_dqn_act(const DqnActArgs& a, hipStream_t s) {
    dim3 grid((unsigned)((a.E + 255) / 256), (unsigned)a.U);
    hipLaunchKernelGGL(k_dqn_act, grid, dim3(256), dqn_act_lds(a.q), s, a);
    return hipGetLastError();
}

hipError_t launch_dqn_grad(const DqnGradArgs& a, const DqnReduceArgs& r, hipStream_t s) {
    hipLaunchKernelGGL(k_dqn_grad, dim3((unsigned)r.nblk, (unsigned)a.q.G), dim3(256), dqn_grad_lds(a.q, a.xpitch), s,
                       a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_dqn_reduce, dim3((unsigned)((r.P + 255) / 256), (unsigned)a.q.G), dim3(256), 0, s, r);
    return hipGetLastError();
}

}  // namespace ms
